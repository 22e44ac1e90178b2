"""Batched BSDF models over device memory -- the Python face of the HIP backbone.

Mirrors the reference's runtime model handle (bsdf_ptr, include/bbm/bsdf_ptr.h:21-165, exposed
to Python as BsdfPtr with eval / sample / pdf / reflectance, include/python/py_core.h:106-112),
but every call takes N direction pairs at once instead of one:

  * directions: a float32 CUDA tensor of shape (3, N) (rows x, y, z -- SoA) or a 3-tuple of
    1-D float32 CUDA tensors;
  * component / unit: bsdf_flag / unit_t, uniform per call (include/bbm/bsdf_flag.h,
    include/bbm/unit.h);
  * mask: optional bool/uint8 tensor of N lanes (the reference's `Mask mask=true`).

All work runs in libbbm_hip (hand-written gfx950 kernels) on the current torch stream; this
module only allocates outputs and passes pointers.  There is no CPU fallback.
"""
import copy
import ctypes
import enum
import re

import numpy as np

from . import _lib
from .models import AGGREGATES, ATTRIBUTES, aggregate_key, attr_size, nparams, to_string


class bsdf_flag(enum.IntFlag):
    """include/bbm/bsdf_flag.h:21-27"""
    None_ = 0
    Diffuse = 1
    Specular = 2
    All = 3


class unit_t(enum.IntEnum):
    """include/bbm/unit.h:20-24"""
    Radiance = 0
    Importance = 1


class BsdfSample:
    """bsdfsample (include/bbm/bsdfsample.h:20-25), batched: direction (3, N), pdf (N,), flag (N,)."""

    def __init__(self, direction, pdf, flag):
        self.direction, self.pdf, self.flag = direction, pdf, flag


def _torch():
    import torch
    return torch


def _is_f64(t):
    """True if the direction rows are float64 (the doubleRGB configuration)."""
    torch = _torch()
    rows = list(t) if isinstance(t, (tuple, list)) else [t]
    return bool(rows) and isinstance(rows[0], torch.Tensor) and rows[0].dtype == torch.float64


def _soa(t, n=None, what="direction", dtype=None):
    """Return (x_ptr, y_ptr, z_ptr, n) for a (3, N) tensor or a tuple of three 1-D tensors of `dtype`
    (float32 unless given)."""
    torch = _torch()
    dtype = torch.float32 if dtype is None else dtype
    if isinstance(t, (tuple, list)):
        rows = list(t)
    else:
        if t.dim() != 2 or t.shape[0] != 3:
            raise ValueError(f"{what}: expected a (3, N) tensor, got {tuple(t.shape)}")
        rows = [t[0], t[1], t[2]]
    for r in rows:
        if not isinstance(r, torch.Tensor) or r.dtype != dtype or not r.is_cuda:
            raise TypeError(f"{what}: expected {str(dtype).replace('torch.', '')} CUDA tensors")
        if r.dim() != 1 or r.stride(0) != 1:
            raise ValueError(f"{what}: rows must be contiguous 1-D tensors")
    m = rows[0].numel()
    if any(r.numel() != m for r in rows):
        raise ValueError(f"{what}: x/y/z lengths differ")
    if n is not None and m != n:
        raise ValueError(f"{what}: expected {n} elements, got {m}")
    return rows[0].data_ptr(), rows[1].data_ptr(), rows[2].data_ptr(), m


def _mask_ptr(mask, n):
    if mask is None:
        return None, None
    torch = _torch()
    if mask.dtype == torch.bool:
        mask = mask.view(torch.uint8)
    if mask.dtype != torch.uint8 or not mask.is_cuda or mask.numel() != n:
        raise TypeError("mask: expected a bool/uint8 CUDA tensor with one entry per pair")
    mask = mask.contiguous()
    return mask.data_ptr(), mask


def _out_rows(t, rows, n, device, what, dtype=None):
    """Validate a caller-supplied output buffer before its row pointers reach a kernel: float32 (or `dtype`), on
    the inputs' device, shape (rows, n) (or (n,) for rows == 0) with every row contiguous."""
    torch = _torch()
    dtype = torch.float32 if dtype is None else dtype
    if not isinstance(t, torch.Tensor) or t.dtype != dtype:
        raise TypeError(f"{what}: expected a {str(dtype).replace('torch.', '')} CUDA tensor")
    if not t.is_cuda or t.device != device:
        raise ValueError(f"{what}: must live on {device}, got {t.device}")
    shape = (n,) if rows == 0 else (rows, n)
    if tuple(t.shape) != shape:
        raise ValueError(f"{what}: expected shape {shape}, got {tuple(t.shape)}")
    if t.stride(-1) != 1:
        raise ValueError(f"{what}: rows must be contiguous")
    return t


def _stream_ptr(stream):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _on_stream(stream, *tensors):
    """Tensors allocated here (outputs, the mask copy) but used by a launch on a stream other than the current
    one: tell the caching allocator, so their memory is not reused before that stream has run the kernel."""
    if stream is None:
        return
    torch = _torch()
    if stream == torch.cuda.current_stream():
        return
    for t in tensors:
        if t is not None:
            t.record_stream(stream)


def model_names():
    """Models available in the loaded HIP library (BBM_EXPORT_BSDFMODEL registry equivalent)."""
    lib = _lib.load()
    return [lib.bbm_hip_model_name(i).decode() for i in range(lib.bbm_hip_num_models())]


def _model_params(model_id, which):
    lib = _lib.load()
    k = _lib.check(lib.bbm_hip_model_nparams(model_id))
    buf = (ctypes.c_float * max(k, 1))()
    _lib.check(lib.bbm_hip_model_params(model_id, which, buf, k))
    return np.array(buf[:k], dtype=np.float32)


class BsdfModel:
    """One parameterised BSDF model, evaluated in batches on the GPU."""

    def __init__(self, name, *args, **kwargs):
        lib = _lib.load()
        if name not in ATTRIBUTES and name not in AGGREGATES:
            raise ValueError(f"unknown BSDF model: {name}")
        mid = lib.bbm_hip_model_id(name.encode())
        if mid < 0:
            raise _lib.BackboneError(mid, f"model {name} is not available in libbbm_hip")
        self.name = name
        self.model_id = mid
        self._params = _model_params(mid, 0)
        if name in AGGREGATES:
            # Aggregate(child, child): children given as models (aggregatemodel.h:33, aggregate() :232-233)
            if kwargs or (args and len(args) != len(AGGREGATES[name])):
                raise TypeError(f"{name}: expected {len(AGGREGATES[name])} child models")
            k = 0
            for c, child in zip(AGGREGATES[name], args):
                if child.name != c:
                    raise TypeError(f"{name}: expected a {c} child, got {child.name}")
                self._params[k:k + child._params.size] = child._params
                k += child._params.size
            return
        layout = ATTRIBUTES[name]
        if len(args) > len(layout):
            raise TypeError(f"{name}: too many positional attributes")
        values = dict(zip([a for a, _ in layout], args))
        for k, v in kwargs.items():
            if k not in dict(layout):
                raise TypeError(f"{name}: unknown attribute '{k}'")
            if k in values:
                raise TypeError(f"{name}: attribute '{k}' given twice")
            values[k] = v
        for k, v in values.items():
            self.set_attribute(k, v)

    @property
    def runtime(self):
        """A fused Aggregate(A, B) evaluated as the reference's runtime aggregatebsdf (what fromString / bsdf_import
        build, include/bbm/aggregatebsdf.h) rather than as aggregatemodel<A, B>: the model id carries
        BBM_HIP_RUNTIME_AGGREGATE."""
        return self.model_id >= 0 and bool(self.model_id & _lib.RUNTIME_AGGREGATE)

    # ---------------------------------------------------------------- attributes
    def _slot(self, attr):
        k = 0
        for a, shape in ATTRIBUTES[self.name]:
            if a == attr:
                return k, shape
            k += attr_size(shape)
        raise KeyError(attr)

    def set_attribute(self, attr, value):
        k, shape = self._slot(attr)
        n = attr_size(shape)
        src = np.asarray(value, dtype=np.float64).reshape(-1)
        with np.errstate(over="ignore"):
            v = src.astype(np.float32)
        if np.any(np.isfinite(src) & ~np.isfinite(v)):
            # the reference's string conversion refuses a value beyond the float range (std::out_of_range)
            raise ValueError(f"{self.name}.{attr}: value out of the float range: {src[np.isfinite(src) & ~np.isfinite(v)]}")
        if v.size == 1 and n > 1:      # a scalar broadcasts over an RGB / Vec2d attribute
            v = np.repeat(v, n)
        if v.size != n:
            raise ValueError(f"{self.name}.{attr}: expected {n} values, got {v.size}")
        self._params[k:k + n] = v

    def attribute(self, attr):
        k, shape = self._slot(attr)
        v = self._params[k:k + attr_size(shape)].copy()
        return v[0] if shape == () else v.reshape(shape)

    def parameter_values(self, flag=None):
        """Flat parameter vector (bbm::parameter_values, include/bbm/bsdf_enumerate.h:103-131).
        flag=None: every parameter (the layout the kernels take, Dependent ones included);
        flag=bsdf_attr bits: only the parameters whose attribute flags intersect it (the reference's
        default bsdf_attr::All = 0x0F leaves out Dependent attributes)."""
        if flag is None:
            return self._params.copy()
        return self._params[self.parameter_indices(flag)].copy()

    def parameter_attrs(self):
        """Per-parameter bsdf_attr flags (bbm_hip_model_param_attrs)."""
        lib = _lib.load()
        k = self._params.size
        buf = (ctypes.c_uint32 * max(k, 1))()
        _lib.check(lib.bbm_hip_model_param_attrs(self.model_id, buf, k))
        return np.array(buf[:k], dtype=np.uint32)

    def parameter_indices(self, flag=0x0F):
        """Indices into the full parameter vector selected by parameter_values(flag)."""
        return np.nonzero(self.parameter_attrs() & np.uint32(flag))[0]

    def children(self):
        """Aggregate: the child models (copies); otherwise []."""
        if self.name not in AGGREGATES:
            return []
        out, k = [], 0
        for c in AGGREGATES[self.name]:
            m = BsdfModel(c)
            m._params[:] = self._params[k:k + m._params.size]
            k += m._params.size
            out.append(m)
        return out

    def set_parameter_values(self, values):
        v = np.asarray(values, dtype=np.float32).reshape(-1)
        if v.size != self._params.size:
            raise ValueError(f"{self.name}: expected {self._params.size} parameters, got {v.size}")
        self._params[:] = v

    def parameter_default_values(self):
        return _model_params(self.model_id, 0)

    def parameter_lower_bound(self):
        return _model_params(self.model_id, 1)

    def parameter_upper_bound(self):
        return _model_params(self.model_id, 2)

    def __str__(self):
        return to_string(self.name, self._params)

    __repr__ = __str__

    # ---------------------------------------------------------------- batched evaluation
    def _call_id(self, exact):
        """The model id for one call: exact=None follows set_exact_subnormals (the process-wide default), True / False
        force exact / default mode for this call only (BBM_HIP_CALL_EXACT / BBM_HIP_CALL_DEFAULT, re-entrant)."""
        if exact is None:
            return self.model_id
        return self.model_id | (_lib.CALL_EXACT if exact else _lib.CALL_DEFAULT)

    def _pptr(self):
        return self._params.ctypes.data_as(ctypes.c_void_p)

    def has_f64(self):
        """True if the model has doubleRGB kernels (bbm_hip_model_has_f64)."""
        return _lib.check(_lib.load().bbm_hip_model_has_f64(self.model_id)) == 1

    def _params_f64(self, params64):
        if params64 is None:
            return np.ascontiguousarray(self._params, dtype=np.float64)
        v = np.ascontiguousarray(params64, dtype=np.float64).reshape(-1)
        if v.size != self._params.size:
            raise ValueError(f"{self.name}: expected {self._params.size} parameters, got {v.size}")
        return v

    def _eval_pdf_f64(self, in_, out, component, unit, mask, rgb, pdf, stream, params64):
        """doubleRGB (Value = double): float64 directions -> float64 eval RGB and pdf (bbm_hip_eval_pdf_f64).
        Parameters: params64 if given, else the model's (float) parameter vector widened to double."""
        torch = _torch()
        f64 = torch.float64
        ix, iy, iz, n = _soa(in_, what="in", dtype=f64)
        ox, oy, oz, _ = _soa(out, n, what="out", dtype=f64)
        mptr, _keep = _mask_ptr(mask, n)
        dev = torch.device("cuda", torch.cuda.current_device())
        rgb = torch.empty((3, n), dtype=f64, device=dev) if rgb is None else _out_rows(rgb, 3, n, dev, "rgb", f64)
        pdf = torch.empty((n,), dtype=f64, device=dev) if pdf is None else _out_rows(pdf, 0, n, dev, "pdf", f64)
        p = self._params_f64(params64)
        _on_stream(stream, _keep, rgb, pdf)
        _lib.check(_lib.load().bbm_hip_eval_pdf_f64(
            self.model_id, p.ctypes.data_as(ctypes.c_void_p), p.size, ix, iy, iz, ox, oy, oz, mptr, n, int(component),
            int(unit), rgb[0].data_ptr(), rgb[1].data_ptr(), rgb[2].data_ptr(), pdf.data_ptr(), _stream_ptr(stream)))
        return rgb, pdf

    def eval_pdf(self, in_, out, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, *,
                 rgb=None, pdf=None, stream=None, mode=3, params64=None, exact=None):
        torch = _torch()
        if _is_f64(in_):
            rgb, pdf = self._eval_pdf_f64(in_, out, component, unit, mask, rgb if mode & 1 else None,
                                          pdf if mode & 2 else None, stream, params64)
            return (rgb if mode & 1 else None), (pdf if mode & 2 else None)
        ix, iy, iz, n = _soa(in_, what="in")
        ox, oy, oz, _ = _soa(out, n, what="out")
        mptr, _keep = _mask_ptr(mask, n)
        dev = torch.device("cuda", torch.cuda.current_device())
        if mode & 1:
            rgb = torch.empty((3, n), dtype=torch.float32, device=dev) if rgb is None else \
                _out_rows(rgb, 3, n, dev, "rgb")
        if mode & 2:
            pdf = torch.empty((n,), dtype=torch.float32, device=dev) if pdf is None else \
                _out_rows(pdf, 0, n, dev, "pdf")
        lib = _lib.load()
        s = _stream_ptr(stream)
        _on_stream(stream, _keep, rgb, pdf)
        mid = self._call_id(exact)
        if mode == 3:
            rc = lib.bbm_hip_eval_pdf(mid, self._pptr(), self._params.size, ix, iy, iz, ox, oy, oz, mptr, n,
                                      int(component), int(unit), rgb[0].data_ptr(), rgb[1].data_ptr(),
                                      rgb[2].data_ptr(), pdf.data_ptr(), s)
        elif mode == 1:
            rc = lib.bbm_hip_eval(mid, self._pptr(), self._params.size, ix, iy, iz, ox, oy, oz, mptr, n,
                                  int(component), int(unit), rgb[0].data_ptr(), rgb[1].data_ptr(), rgb[2].data_ptr(), s)
        else:
            rc = lib.bbm_hip_pdf(mid, self._pptr(), self._params.size, ix, iy, iz, ox, oy, oz, mptr, n,
                                 int(component), int(unit), pdf.data_ptr(), s)
        _lib.check(rc)
        return rgb, pdf

    def eval(self, in_, out, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, **kw):
        """Spectrum eval(in, out, component, unit, mask) for N pairs -> (3, N) RGB."""
        return self.eval_pdf(in_, out, component, unit, mask, mode=1, **kw)[0]

    def pdf(self, in_, out, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, **kw):
        """Value pdf(in, out, component, unit, mask) for N pairs -> (N,)."""
        return self.eval_pdf(in_, out, component, unit, mask, mode=2, **kw)[1]

    def sample(self, out, xi, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, *, stream=None,
               params64=None, exact=None):
        """BsdfSample sample(out, xi, component, unit, mask) for N (out, xi) -> BsdfSample (float64 out / xi: the
        doubleRGB kernels, float64 direction and pdf).  exact: as eval_pdf."""
        torch = _torch()
        f64 = _is_f64(out)
        dt = torch.float64 if f64 else torch.float32
        ox, oy, oz, n = _soa(out, what="out", dtype=dt)
        if isinstance(xi, (tuple, list)):
            x0, x1 = xi
        else:
            if xi.dim() != 2 or xi.shape[0] != 2:
                raise ValueError("xi: expected a (2, N) tensor")
            x0, x1 = xi[0], xi[1]
        for x in (x0, x1):
            if x.dtype != dt or not x.is_cuda or x.numel() != n or x.stride(0) != 1:
                raise TypeError(f"xi: expected {str(dt).replace('torch.', '')} CUDA rows with one entry per direction")
        mptr, _keep = _mask_ptr(mask, n)
        dev = x0.device
        d = torch.empty((3, n), dtype=dt, device=dev)
        p = torch.empty((n,), dtype=dt, device=dev)
        f = torch.empty((n,), dtype=torch.int32, device=dev)
        _on_stream(stream, _keep, d, p, f)
        lib = _lib.load()
        if f64:
            prm = self._params_f64(params64)
            fn, pp, npar = lib.bbm_hip_sample_f64, prm.ctypes.data_as(ctypes.c_void_p), prm.size
        else:
            fn, pp, npar = lib.bbm_hip_sample, self._pptr(), self._params.size
        _lib.check(fn(self._call_id(exact), pp, npar, ox, oy, oz, x0.data_ptr(), x1.data_ptr(), mptr, n, int(component),
                      int(unit), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), p.data_ptr(), f.data_ptr(),
                      _stream_ptr(stream)))
        return BsdfSample(d, p, f)

    def reflectance(self, out, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, *, stream=None,
                    params64=None, exact=None):
        """Spectrum reflectance(out, component, unit, mask) for N directions -> (3, N) RGB (float64 directions:
        the doubleRGB kernels, float64 RGB)."""
        torch = _torch()
        if _is_f64(out):
            ox, oy, oz, n = _soa(out, what="out", dtype=torch.float64)
            mptr, _keep = _mask_ptr(mask, n)
            dev = (out[0] if isinstance(out, (tuple, list)) else out).device
            rgb = torch.empty((3, n), dtype=torch.float64, device=dev)
            p = self._params_f64(params64)
            _on_stream(stream, _keep, rgb)
            _lib.check(_lib.load().bbm_hip_reflectance_f64(
                self.model_id, p.ctypes.data_as(ctypes.c_void_p), p.size, ox, oy, oz, mptr, n, int(component),
                int(unit), rgb[0].data_ptr(), rgb[1].data_ptr(), rgb[2].data_ptr(), _stream_ptr(stream)))
            return rgb
        ox, oy, oz, n = _soa(out, what="out")
        mptr, _keep = _mask_ptr(mask, n)
        dev = (out[0] if isinstance(out, (tuple, list)) else out).device
        rgb = torch.empty((3, n), dtype=torch.float32, device=dev)
        _on_stream(stream, _keep, rgb)
        lib = _lib.load()
        _lib.check(lib.bbm_hip_reflectance(self._call_id(exact), self._pptr(), self._params.size, ox, oy, oz, mptr, n,
                                           int(component), int(unit), rgb[0].data_ptr(), rgb[1].data_ptr(),
                                           rgb[2].data_ptr(), _stream_ptr(stream)))
        return rgb


# ------------------------------------------------------------------------- string import

_TOKEN = re.compile(r"\s*([A-Za-z_][A-Za-z0-9_]*|[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?|[()\[\],=])")


def _tokenize(s):
    pos, out = 0, []
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise ValueError(f"cannot parse BSDF string at: {s[pos:]!r}")
        out.append(m.group(1))
        pos = m.end()
    return out


def _parse_value(tok, i):
    if tok[i] == "[":
        vals, i = [], i + 1
        while tok[i] != "]":
            v, i = _parse_value(tok, i)
            vals.append(v)
            if tok[i] == ",":
                i += 1
        return vals, i + 1
    return float(tok[i]), i + 1


def _parse_model(tok, i, s):
    """Parse `Name(...)` starting at tok[i]; returns (model, next index)."""
    name = tok[i]
    if name == "Aggregate":
        # Aggregate(child, child) (aggregatemodel.h:184-212)
        if i + 1 >= len(tok) or tok[i + 1] != "(":
            raise ValueError(f"malformed BSDF string: {s!r}")
        kids, i = [], i + 2
        while tok[i] != ")":
            m, i = _parse_model(tok, i, s)
            kids.append(m)
            if tok[i] == ",":
                i += 1
        # the runtime aggregate: fromString<bsdf_ptr> maps "Aggregate" to aggregatebsdf (bsdf_string_convert.h:59)
        return Aggregate(*kids, runtime=True), i + 1
    if name not in ATTRIBUTES:
        raise ValueError(f"unknown BSDF model: {name}")
    m = BsdfModel(name)
    if i + 1 >= len(tok) or tok[i + 1] != "(":
        return m, i + 1
    i, layout, pos_idx = i + 2, [a for a, _ in ATTRIBUTES[name]], 0
    while tok[i] != ")":
        if i + 1 < len(tok) and tok[i + 1] == "=":
            attr = tok[i]
            v, i = _parse_value(tok, i + 2)
        else:
            attr = layout[pos_idx]
            v, i = _parse_value(tok, i)
        pos_idx += 1
        m.set_attribute(attr, np.asarray(v, dtype=np.float64))
        if tok[i] == ",":
            i += 1
    return m, i + 1


def fromString(s):
    """Construct a model from its bbm::toString form, e.g. 'CookTorrance(albedo = [0.5, 0.5, 0.5],
    roughness = 0.1, eta = 1.3)' or 'Aggregate(Lambertian(...), Bagher(...))'
    (bsdf_string_convert.h:52-82 / bsdf_import.h:22-26).  Attributes may appear in any order;
    missing ones keep their defaults."""
    mm = re.fullmatch(r'\s*Merl\(\s*"([^"]*)"\s*\)\s*', s)
    if mm:          # merl_data's string form, Merl("filename") (merl.h:60, :161-164)
        from .merl import Merl
        return Merl(mm.group(1))
    tok = _tokenize(s)
    m, i = _parse_model(tok, 0, s)
    if i != len(tok):
        raise ValueError(f"malformed BSDF string: {s!r}")
    return m


bsdf_import = fromString


def parse_model(s):
    """fromString through the library's own C-ABI parser (bbm_hip_parse_model_tree, the restatement of the
    reference's runtime fromString, bsdf_string_convert.h:52-85, that FFI callers use): the same models as
    fromString, built from the parser's preorder tree -- registry leaves (a fused runtime aggregate keeps its
    BBM_HIP_RUNTIME_AGGREGATE id), BBM_HIP_AGGREGATE_BSDF nodes as runtime AggregateModels."""
    lib = _lib.load()
    cap_nodes, cap_params = 256, 1 << 14
    ids, nk, npar = (ctypes.c_int * cap_nodes)(), (ctypes.c_int * cap_nodes)(), (ctypes.c_int * cap_nodes)()
    buf = np.zeros(cap_params, np.float32)
    k = _lib.check(lib.bbm_hip_parse_model_tree(s.encode(), ids, nk, buf.ctypes.data_as(ctypes.c_void_p), npar,
                                                 cap_nodes, cap_params))
    pos = [0, 0]            # next node, next parameter

    def build():
        i = pos[0]
        pos[0] += 1
        if ids[i] == _lib.AGGREGATE_BSDF:
            return AggregateModel(*[build() for _ in range(nk[i])], runtime=True)
        mid = ids[i]
        m = BsdfModel(lib.bbm_hip_model_name(mid & ~_lib.RUNTIME_AGGREGATE).decode())
        m.set_parameter_values(buf[pos[1]:pos[1] + npar[i]])
        pos[1] += npar[i]
        m.model_id = mid
        return m
    m = build()
    assert pos[0] == k
    return m


def _copy_model(m):
    """A copy of a model for an aggregate (aggregatemodel_base copies its children, aggregatemodel.h:34): same
    class, own parameter vector, and every other attribute shared -- a Merl child keeps the reference to the
    device table its parameters point to."""
    if isinstance(m, AggregateModel):
        return AggregateModel(*m._children, runtime=m.runtime)
    c = copy.copy(m)
    c._params = m._params.copy()
    return c


class AggregateModel:
    """aggregatemodel<MODELS...> (include/bsdfmodel/aggregatemodel.h:22-222) of any >= 2 models -- single models,
    Merl, fused aggregates, or composed aggregates again (aggregatemodel_base takes any bsdfmodel child, :22) --
    evaluated by composing the children's kernels (bbm_hip_aggregate_*, bbm_amd/csrc/composite.hip): eval /
    reflectance = the children's sum (right fold), pdf = their reflectance-weighted mixture, sample = the
    reference's child selection on xi0; a nested aggregate is one child with its own eval / pdf / sample /
    reflectance.  The published fits' form Aggregate(Lambertian, X) has fused kernels instead (Aggregate(...)
    picks them).  Parameters are the children's vectors in order (reflection order of the base classes).
    float32 tensors evaluate in floatRGB, float64 tensors in doubleRGB (every leaf needs doubleRGB kernels)."""

    def __init__(self, *children, runtime=False):
        if len(children) < 2:
            raise ValueError("an aggregate needs at least two child models")
        for c in children:
            if not isinstance(c, (BsdfModel, AggregateModel)):
                raise TypeError("aggregate children must be models (BsdfModel, Merl or AggregateModel)")
        self._children = [_copy_model(c) for c in children]
        self.name = aggregate_key([c.name for c in children])
        # runtime: the reference's aggregatebsdf (left folds, per-term pdf quotients, no sample unless the weights
        # sum to > eps; include/bbm/aggregatebsdf.h), what fromString builds; else aggregatemodel<...>
        self.runtime = bool(runtime)

    def children(self):
        return [_copy_model(c) for c in self._children]

    def parameter_values(self, flag=None):
        return np.concatenate([c.parameter_values(flag) for c in self._children])

    # the reference enumerates an aggregate's attributes child by child (bsdf_enumerate.h over the base classes)
    def parameter_attrs(self):
        return np.concatenate([c.parameter_attrs() for c in self._children])

    def parameter_indices(self, flag=0x0F):
        return np.nonzero(self.parameter_attrs() & np.uint32(flag))[0]

    def parameter_default_values(self):
        return np.concatenate([c.parameter_default_values() for c in self._children])

    def parameter_lower_bound(self):
        return np.concatenate([c.parameter_lower_bound() for c in self._children])

    def parameter_upper_bound(self):
        return np.concatenate([c.parameter_upper_bound() for c in self._children])

    def set_parameter_values(self, values):
        v = np.asarray(values, dtype=np.float32).reshape(-1)
        sizes = [c.parameter_values().size for c in self._children]
        if v.size != sum(sizes):
            raise ValueError(f"{self.name}: expected {sum(sizes)} parameters, got {v.size}")
        k = 0
        for c, n in zip(self._children, sizes):
            c.set_parameter_values(v[k:k + n])
            k += n

    def __str__(self):
        return "Aggregate(" + ", ".join(str(c) for c in self._children) + ")"

    __repr__ = __str__

    def has_f64(self):
        return all(c.has_f64() for c in self._children)

    def _desc(self, f64=False, params=None):
        """ctypes bbm_hip_child(_f64) tree: (array, count, keep-alive list of the arrays and parameter buffers it
        points to).  An aggregatemodel passes its children (count >= 2); a runtime aggregate passes its root node
        (count 1, BBM_HIP_AGGREGATE_BSDF), the only way to give the top level aggregatebsdf semantics.  Nested
        aggregates are AGGREGATE / AGGREGATE_BSDF nodes.  params: the flat parameter vector to use instead of the
        children's own (the leaves in preorder)."""
        keep = []
        kind = _lib.ChildF64 if f64 else _lib.Child
        flat = None if params is None else np.asarray(params).reshape(-1)
        off = [0]

        def leaf_params(c):
            if flat is None:
                return c._params
            k = c._params.size
            off[0] += k
            return flat[off[0] - k:off[0]]

        def node(a, c):
            if isinstance(c, AggregateModel):
                sub = build(c._children)
                a.model_id, a.params, a.nparams = (_lib.AGGREGATE_BSDF if c.runtime else _lib.AGGREGATE), None, 0
                a.children, a.nchildren = ctypes.cast(sub, ctypes.c_void_p), len(c._children)
            else:
                c._pptr()          # a Merl child checks its table's device here
                p = np.ascontiguousarray(leaf_params(c), dtype=np.float64 if f64 else np.float32)
                keep.append(p)
                a.model_id, a.params, a.nparams = c.model_id, p.ctypes.data, p.size
                a.children, a.nchildren = None, 0

        def build(kids):
            arr = (kind * len(kids))()
            keep.append(arr)
            for a, c in zip(arr, kids):
                node(a, c)
            return arr
        if self.runtime:
            root = (kind * 1)()
            keep.append(root)
            node(root[0], self)
            return root, 1, keep
        return build(self._children), len(self._children), keep

    def eval_pdf(self, in_, out, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, *,
                 rgb=None, pdf=None, stream=None, mode=3):
        torch = _torch()
        f64 = _is_f64(in_)
        dt = torch.float64 if f64 else torch.float32
        ix, iy, iz, n = _soa(in_, what="in", dtype=dt)
        ox, oy, oz, _ = _soa(out, n, what="out", dtype=dt)
        mptr, _keep = _mask_ptr(mask, n)
        dev = torch.device("cuda", torch.cuda.current_device())
        if mode & 1:
            rgb = torch.empty((3, n), dtype=dt, device=dev) if rgb is None else _out_rows(rgb, 3, n, dev, "rgb", dt)
        if mode & 2:
            pdf = torch.empty((n,), dtype=dt, device=dev) if pdf is None else _out_rows(pdf, 0, n, dev, "pdf", dt)
        _on_stream(stream, _keep, rgb, pdf)
        d, nd, _kd = self._desc(f64)
        fn = _lib.load().bbm_hip_aggregate_eval_pdf_f64 if f64 else _lib.load().bbm_hip_aggregate_eval_pdf
        _lib.check(fn(d, nd, ix, iy, iz, ox, oy, oz, mptr, n, int(component), int(unit),
                      rgb[0].data_ptr() if mode & 1 else None, rgb[1].data_ptr() if mode & 1 else None,
                      rgb[2].data_ptr() if mode & 1 else None, pdf.data_ptr() if mode & 2 else None,
                      _stream_ptr(stream)))
        return rgb, pdf

    eval = BsdfModel.eval
    pdf = BsdfModel.pdf

    def sample(self, out, xi, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, *, stream=None):
        torch = _torch()
        f64 = _is_f64(out)
        dt = torch.float64 if f64 else torch.float32
        ox, oy, oz, n = _soa(out, what="out", dtype=dt)
        x0, x1 = (xi if isinstance(xi, (tuple, list)) else (xi[0], xi[1]))
        for x in (x0, x1):
            if x.dtype != dt or not x.is_cuda or x.numel() != n or x.stride(0) != 1:
                raise TypeError(f"xi: expected {str(dt).replace('torch.', '')} CUDA rows with one entry per direction")
        mptr, _keep = _mask_ptr(mask, n)
        dev = x0.device
        d = torch.empty((3, n), dtype=dt, device=dev)
        p = torch.empty((n,), dtype=dt, device=dev)
        f = torch.empty((n,), dtype=torch.int32, device=dev)
        _on_stream(stream, _keep, d, p, f)
        desc, nd, _kd = self._desc(f64)
        fn = _lib.load().bbm_hip_aggregate_sample_f64 if f64 else _lib.load().bbm_hip_aggregate_sample
        _lib.check(fn(desc, nd, ox, oy, oz, x0.data_ptr(), x1.data_ptr(), mptr, n, int(component),
                      int(unit), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), p.data_ptr(), f.data_ptr(),
                      _stream_ptr(stream)))
        return BsdfSample(d, p, f)

    def reflectance(self, out, component=bsdf_flag.All, unit=unit_t.Radiance, mask=None, *, stream=None):
        torch = _torch()
        f64 = _is_f64(out)
        dt = torch.float64 if f64 else torch.float32
        ox, oy, oz, n = _soa(out, what="out", dtype=dt)
        mptr, _keep = _mask_ptr(mask, n)
        dev = (out[0] if isinstance(out, (tuple, list)) else out).device
        rgb = torch.empty((3, n), dtype=dt, device=dev)
        _on_stream(stream, _keep, rgb)
        desc, nd, _kd = self._desc(f64)
        fn = _lib.load().bbm_hip_aggregate_reflectance_f64 if f64 else _lib.load().bbm_hip_aggregate_reflectance
        _lib.check(fn(desc, nd, ox, oy, oz, mptr, n, int(component), int(unit), rgb[0].data_ptr(),
                      rgb[1].data_ptr(), rgb[2].data_ptr(), _stream_ptr(stream)))
        return rgb


def tree_desc(model, f64=False):
    """Any model as a bbm_hip_child(_f64) tree for the *_tree entry points (bbm_hip_loss_tree, bbm_hip_check_tree):
    (array, count, keep-alive list).  A single model (or fused aggregate, Merl) is one leaf node; an AggregateModel
    its children or its runtime root node (AggregateModel._desc)."""
    if isinstance(model, AggregateModel):
        return model._desc(f64)
    kind = _lib.ChildF64 if f64 else _lib.Child
    arr = (kind * 1)()
    p = model._pptr() if not f64 else None
    params = np.ascontiguousarray(model._params, dtype=np.float64) if f64 else model._params
    arr[0].model_id, arr[0].params, arr[0].nparams = model.model_id, params.ctypes.data, params.size
    arr[0].children, arr[0].nchildren = None, 0
    return arr, 1, [arr, params, p]


def Aggregate(*children, fused=True, runtime=False):
    """aggregate(models...) (aggregatemodel.h:232-233): the fused kernel for the published fits' form
    Aggregate(Lambertian, X) where one is registered (fused=False forces the composed path), otherwise an
    AggregateModel over the children's own kernels.

    Note: this mirrors the C++ template aggregate() (aggregatemodel<...>), NOT the reference's Python binding
    bbm.Aggregate (include/python/py_core.h:116-123), which builds the runtime aggregatebsdf of bsdf_ptrs.  The two
    differ in the pdf's rounding (inner product / sum here, per-term there) and in sampling (here a child is sampled
    even when the weights sum below eps).  Scripts ported from the reference's Python API get the binding's
    semantics with runtime=True, or with fromString("Aggregate(...)"), which returns runtime aggregates like
    bsdf_import does."""
    key = aggregate_key([c.name for c in children])
    if fused and key in AGGREGATES and all(isinstance(c, BsdfModel) for c in children):
        m = BsdfModel(key, *children)
        if runtime:
            m.model_id |= _lib.RUNTIME_AGGREGATE
        return m
    return AggregateModel(*children, runtime=runtime)


def _make_ctor(name):
    def ctor(*args, **kwargs):
        return BsdfModel(name, *args, **kwargs)
    ctor.__name__ = name
    if name in ATTRIBUTES:
        ctor.__doc__ = f"Constructs: {name}({', '.join(a for a, _ in ATTRIBUTES[name])}) -- {nparams(name)} parameters"
    return ctor


def scratch_trim():
    """Return the library's idle device scratch (per-launch temporaries of composed aggregates and tabulated
    samplers) to the device (bbm_hip_scratch_trim); returns the bytes freed."""
    return int(_lib.load().bbm_hip_scratch_trim())


def scratch_trim_captured():
    """Free the scratch blocks that HIP-graph captures of library calls hold (bbm_hip_scratch_trim_captured): only
    once every such graph is destroyed.  Returns the bytes freed."""
    return int(_lib.load().bbm_hip_scratch_trim_captured())


def scratch_bytes():
    """Device bytes the library's scratch pool currently holds (bbm_hip_scratch_bytes)."""
    return int(_lib.load().bbm_hip_scratch_bytes())


def set_exact_subnormals(on):
    """Exact-subnormal mode of the Beckmann microfacet models' eval / pdf kernels (bbm_hip_set_exact_subnormals,
    process-wide): on, the quotients a subnormal intermediate can reach round on the subnormal grid as the
    reference's IEEE divisions do, and CookTorrance & co. return the reference's floats bit for bit (+3.6-4.3 % kernel
    time on the headline); off (default), outputs below ~1e-30 may differ in the last bit.  Returns the previous
    setting."""
    return bool(_lib.load().bbm_hip_set_exact_subnormals(1 if on else 0))


def fill_directions(seed, stream_id, offset, n, mode=0, out=None, stream=None):
    """Counter-based synthetic directions (bbm_hip_fill_directions) -> (3, n) float32 CUDA tensor."""
    torch = _torch()
    if out is None:
        out = torch.empty((3, n), dtype=torch.float32, device=torch.device("cuda", torch.cuda.current_device()))
    lib = _lib.load()
    _lib.check(lib.bbm_hip_fill_directions(seed, stream_id, offset, n, mode, out[0].data_ptr(), out[1].data_ptr(),
                                           out[2].data_ptr(), _stream_ptr(stream)))
    return out
