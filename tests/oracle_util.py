"""Test-side access to the oracle (CPU checkers) and the golden fixtures.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
  * port: oracle/_port/libbbm_port.so -- our C restatement of the native backbone (oracle/port);
  * ref : oracle/_ref/libbbm_ref.so   -- the reference's own headers behind a ctypes shim
          (prebuilt in the build container; absent if it was never built);
  * golden: tests/golden/*.npz written by oracle/gen_golden.py from the reference.
"""
import ctypes
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PORT_LIB = os.path.join(ROOT, "oracle", "_port", "libbbm_port.so")
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libbbm_ref.so")
# the same shim built with the reference's Release flags (-O3, SLP vectorization on): timed by the cpu_baseline legs only
REF_BENCH_LIB = os.path.join(ROOT, "oracle", "_ref", "libbbm_ref_bench.so")

_libs = {}


def _fp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _load(path, prefix):
    if path not in _libs:
        if not os.path.exists(path):
            return None
        lib = ctypes.CDLL(path)
        getattr(lib, prefix + "model_name").restype = ctypes.c_char_p
        _libs[path] = lib
    return _libs[path]


def port():
    return _load(PORT_LIB, "bbmport_")


def ref():
    return _load(REF_LIB, "bbmref_")


def ref_bench():
    """The reference for CPU timing (bench.py / tools/bench_configs.py cpu_baseline): the -O3 Release build, or the
    checker build where it is absent.  Never a checker: g++ 11.4's -O3 SLP miscompiles the He family's D
    (oracle/Makefile, profiles/r06_oracle_slp.txt)."""
    return _load(REF_BENCH_LIB, "bbmref_") or ref()


def port_models():
    lib = port()
    return [lib.bbmport_model_name(i).decode() for i in range(lib.bbmport_num_models())]


def _evalpdf(fn, name, params, din, dout, component, unit, nthreads):
    params = np.ascontiguousarray(params, dtype=np.float32)
    din = np.ascontiguousarray(din, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    n = din.shape[1]
    res = np.zeros((4, n), np.float32)
    rc = fn(name.encode(), _fp(params), params.size, ctypes.c_size_t(n), _fp(din[0]), _fp(din[1]), _fp(din[2]),
            _fp(dout[0]), _fp(dout[1]), _fp(dout[2]), ctypes.c_uint32(component), ctypes.c_uint32(unit), 3,
            _fp(res[0]), _fp(res[1]), _fp(res[2]), _fp(res[3]), nthreads)
    if rc != 0:
        raise KeyError(f"oracle has no model {name} (rc={rc})")
    return res


def port_eval_pdf(name, params, din, dout, component=3, unit=0, nthreads=1):
    """(4, N): eval RGB + pdf from the C restatement."""
    return _evalpdf(port().bbmport_eval_pdf, name, params, din, dout, component, unit, nthreads)


def ref_eval_pdf(name, params, din, dout, component=3, unit=0, nthreads=1):
    """(4, N): eval RGB + pdf from the reference itself (None if the prebuilt shim is absent)."""
    lib = ref()
    if lib is None:
        return None
    return _evalpdf(lib.bbmref_eval_pdf, name, params, din, dout, component, unit, nthreads)


def _sample(fn, name, params, dout, xi, component, unit, nthreads):
    params = np.ascontiguousarray(params, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    xi = np.ascontiguousarray(xi, dtype=np.float32)
    n = dout.shape[1]
    res = np.zeros((4, n), np.float32)
    flag = np.zeros(n, np.uint32)
    rc = fn(name.encode(), _fp(params), params.size, ctypes.c_size_t(n), _fp(dout[0]), _fp(dout[1]), _fp(dout[2]),
            _fp(xi[0]), _fp(xi[1]), ctypes.c_uint32(component), ctypes.c_uint32(unit),
            _fp(res[0]), _fp(res[1]), _fp(res[2]), _fp(res[3]), _fp(flag), nthreads)
    if rc != 0:
        raise KeyError(f"oracle cannot sample model {name} (rc={rc})")
    return res, flag


def port_sample(name, params, dout, xi, component=3, unit=0, nthreads=1):
    return _sample(port().bbmport_sample, name, params, dout, xi, component, unit, nthreads)


def ref_sample(name, params, dout, xi, component=3, unit=0, nthreads=1):
    lib = ref()
    if lib is None:
        return None
    return _sample(lib.bbmref_sample, name, params, dout, xi, component, unit, nthreads)


def ref_reflectance(name, params, dout, component=3, unit=0):
    """(3, N): reflectance(out) from the reference itself."""
    lib = ref()
    params = np.ascontiguousarray(params, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    n = dout.shape[1]
    res = np.zeros((3, n), np.float32)
    rc = lib.bbmref_reflectance(name.encode(), _fp(params), params.size, ctypes.c_size_t(n), _fp(dout[0]),
                                _fp(dout[1]), _fp(dout[2]), ctypes.c_uint32(component), ctypes.c_uint32(unit),
                                _fp(res[0]), _fp(res[1]), _fp(res[2]))
    if rc != 0:
        raise KeyError(f"oracle has no model {name} (rc={rc})")
    return res


def ref_eval_pdf_double(name, params, din, dout, component=3, unit=0, nthreads=1):
    """(4, N) float64: eval RGB + pdf from the reference's doubleRGB configuration (float parameters and directions
    widened to double, as the GPU's f64 path receives them)."""
    lib = ref()
    params = np.ascontiguousarray(params, dtype=np.float32)
    din = np.ascontiguousarray(din, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    n = din.shape[1]
    res = np.zeros((4, n), np.float64)
    rc = lib.bbmref_eval_pdf_double(name.encode(), _fp(params), params.size, ctypes.c_size_t(n), _fp(din[0]),
                                    _fp(din[1]), _fp(din[2]), _fp(dout[0]), _fp(dout[1]), _fp(dout[2]),
                                    ctypes.c_uint32(component), ctypes.c_uint32(unit), 3, _fp(res[0]), _fp(res[1]),
                                    _fp(res[2]), _fp(res[3]), nthreads)
    if rc != 0:
        raise KeyError(f"oracle has no model {name} (rc={rc})")
    return res


def ref_eval_pdf_dd(name, params, din, dout, component=3, unit=0, nthreads=1):
    """(4, N) float64: the reference's doubleRGB eval + pdf at float64 directions."""
    lib = ref()
    params = np.ascontiguousarray(params, dtype=np.float32)
    din = np.ascontiguousarray(din, dtype=np.float64)
    dout = np.ascontiguousarray(dout, dtype=np.float64)
    n = din.shape[1]
    res = np.zeros((4, n), np.float64)
    rc = lib.bbmref_eval_pdf_dd(name.encode(), _fp(params), params.size, ctypes.c_size_t(n), _fp(din[0]), _fp(din[1]),
                                _fp(din[2]), _fp(dout[0]), _fp(dout[1]), _fp(dout[2]), ctypes.c_uint32(component),
                                ctypes.c_uint32(unit), 3, _fp(res[0]), _fp(res[1]), _fp(res[2]), _fp(res[3]), nthreads)
    if rc != 0:
        raise KeyError(f"oracle has no model {name} (rc={rc})")
    return res


def ref_sample_double(name, params, dout, xi, component=3, unit=0, nthreads=1):
    """doubleRGB sample(out, xi) from the reference: ((3, N) float64 direction, (N,) float64 pdf, (N,) flags)."""
    lib = ref()
    params = np.ascontiguousarray(params, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    xi = np.ascontiguousarray(xi, dtype=np.float32)
    n = dout.shape[1]
    d = np.zeros((4, n), np.float64)
    flag = np.zeros(n, np.uint32)
    rc = lib.bbmref_sample_double(name.encode(), _fp(params), params.size, ctypes.c_size_t(n), _fp(dout[0]),
                                  _fp(dout[1]), _fp(dout[2]), _fp(xi[0]), _fp(xi[1]), ctypes.c_uint32(component),
                                  ctypes.c_uint32(unit), _fp(d[0]), _fp(d[1]), _fp(d[2]), _fp(d[3]), _fp(flag), nthreads)
    if rc != 0:
        raise KeyError(f"oracle has no model {name} (rc={rc})")
    return d[:3], d[3], flag


def ref_reflectance_double(name, params, dout, component=3, unit=0):
    """(3, N) float64: reflectance(out) from the reference's doubleRGB configuration."""
    lib = ref()
    params = np.ascontiguousarray(params, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    n = dout.shape[1]
    res = np.zeros((3, n), np.float64)
    rc = lib.bbmref_reflectance_double(name.encode(), _fp(params), params.size, ctypes.c_size_t(n), _fp(dout[0]),
                                       _fp(dout[1]), _fp(dout[2]), ctypes.c_uint32(component), ctypes.c_uint32(unit),
                                       _fp(res[0]), _fp(res[1]), _fp(res[2]))
    if rc != 0:
        raise KeyError(f"oracle has no model {name} (rc={rc})")
    return res


def ref_default_params(name):
    """The reference's default parameter vector of model `name` (All | Dependent, declaration order; nested
    aggregates child by child)."""
    lib = ref()
    buf = np.zeros(256, np.float32)
    k = lib.bbmref_default_params(name.encode(), _fp(buf), 256)
    if k < 0:
        raise KeyError(f"oracle has no model {name}")
    return buf[:k].copy()


def ref_to_string(name, params):
    """bbm::toString of model `name` at `params`, from the reference."""
    lib = ref()
    params = np.ascontiguousarray(params, dtype=np.float32)
    buf = ctypes.create_string_buffer(16384)
    k = lib.bbmref_to_string(name.encode(), _fp(params), params.size, buf, 16384)
    if k < 0:
        raise KeyError(f"oracle has no model {name}")
    return buf.value.decode()


def ref_from_string(name, s):
    """bbm::fromString<name>(s) -> the parameter vector, or None if the reference rejects the string."""
    lib = ref()
    buf = np.zeros(256, np.float32)
    k = lib.bbmref_from_string(name.encode(), s.encode(), _fp(buf), 256)
    return None if k < 0 else buf[:k].copy()


def oracle_models():
    """Models a CPU checker can evaluate on arbitrary inputs: the reference shim if it is present
    (prebuilt in the build container, travels with the tree), else the C restatement."""
    lib = ref()
    if lib is not None:
        return [lib.bbmref_model_name(i).decode() for i in range(lib.bbmref_num_models())]
    return port_models()


def oracle_eval_pdf(name, params, din, dout, component=3, unit=0, nthreads=1):
    if ref() is not None:
        return ref_eval_pdf(name, params, din, dout, component, unit, nthreads)
    return port_eval_pdf(name, params, din, dout, component, unit, nthreads)


def oracle_sample(name, params, dout, xi, component=3, unit=0, nthreads=1):
    if ref() is not None:
        return ref_sample(name, params, dout, xi, component, unit, nthreads)
    return port_sample(name, params, dout, xi, component, unit, nthreads)


# ------------------------------------------------------------------------------ golden

def golden_meta():
    with open(os.path.join(GOLDEN, "models.json")) as f:
        return json.load(f)


def golden_inputs():
    return np.load(os.path.join(GOLDEN, "inputs.npz"))


def golden_model(name):
    return np.load(os.path.join(GOLDEN, name.replace("<", "_").replace(",", "_").replace(">", "") + ".npz"))


# ------------------------------------------------------------------------------ comparison

def rel_err(got, ref):
    """Element-wise relative error; exact agreement (incl. both zero / both NaN) counts as 0."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    same = (got == ref) | (np.isnan(got) & np.isnan(ref))
    err = np.abs(got - ref) / np.maximum(np.abs(ref), np.finfo(np.float32).tiny)
    err[same] = 0.0
    err[np.isnan(err)] = np.inf
    return err


def ulp_diff(got, ref):
    """|ulp distance| between float32 arrays (NaN == NaN counts as 0)."""
    a = np.asarray(got, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(ref, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    d = np.abs(a - b)
    both_nan = np.isnan(np.asarray(got, np.float32)) & np.isnan(np.asarray(ref, np.float32))
    d[both_nan] = 0
    return d


# Parity bar (BASELINE.json north_star), lane by lane, no batch-dependent floor:
#   * every lane whose reference value is a normal float (|ref| >= FLT_MIN):  |gpu - ref| <= 1e-5 |ref|;
#   * lanes whose reference value is subnormal or zero: |gpu - ref| <= 1e-5 FLT_MIN (the same bar, continued
#     below the normal range with the absolute step it has at FLT_MIN: ~83 subnormal ulps);
#   * NaN where the reference is NaN, the same infinity where it is infinite.
# Nothing else is excused here; a test that accepts a lane outside this bar must prove that lane on its own
# (e.g. the reference, given inputs a few ulps away, reproduces the GPU value: test_gpu_parity.py).
REL_TOL = 1e-5
FLT_MIN = float(np.finfo(np.float32).tiny)


def parity_ok(got, ref, rel_tol=REL_TOL):
    """Boolean mask of lanes that meet the bar above."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    with np.errstate(invalid="ignore"):
        tol = rel_tol * np.maximum(np.abs(ref), FLT_MIN)
        ok = (np.abs(got - ref) <= tol) | (got == ref) | (np.isnan(got) & np.isnan(ref))
    return ok


DBL_MIN = float(np.finfo(np.float64).tiny)


def parity_ok_f64(got, ref, rel_tol=REL_TOL):
    """The same bar for doubleRGB outputs: |gpu - ref| <= rel_tol |ref| for every normal double, the absolute step
    rel_tol DBL_MIN below the normal range, NaN for NaN."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    with np.errstate(invalid="ignore"):
        tol = rel_tol * np.maximum(np.abs(ref), DBL_MIN)
        ok = (np.abs(got - ref) <= tol) | (got == ref) | (np.isnan(got) & np.isnan(ref))
    return ok


def rel_err_f64(got, ref):
    """Element-wise relative error of float64 results (exact agreement = 0)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    same = (got == ref) | (np.isnan(got) & np.isnan(ref))
    with np.errstate(invalid="ignore", divide="ignore"):
        err = np.abs(got - ref) / np.maximum(np.abs(ref), DBL_MIN)
    err[same] = 0.0
    err[np.isnan(err)] = np.inf
    return err


def parity_violations(got, ref, rel_tol=REL_TOL):
    return np.nonzero(~parity_ok(got, ref, rel_tol))


def perturb_ulps(a, steps):
    """a (float32) moved by `steps` (integer array, same shape) float steps: the float `steps` positions away in
    the ordered float line (np.nextafter applied |steps| times, vectorised on the bit patterns)."""
    a = np.asarray(a, np.float32)
    b = a.view(np.int32).astype(np.int64)
    key = np.where(b < 0, -(b & 0x7FFFFFFF), b) + np.asarray(steps, np.int64)
    out = np.where(key < 0, (-key) | 0x80000000, key).astype(np.uint32).view(np.float32)
    return out


def explained_by_input_ulps(ref_fn, inputs, got, k=2, trials=48, seed=1234, any_match=False, abs_tol=0.0):
    """Per-lane proof for lanes outside the bar (backward error): True for a lane where every output channel of
    the GPU lies within the bar of -- or between -- the reference's own outputs at inputs whose coordinates are
    each moved by at most k float steps (the unmoved input and `trials - 1` random moves, seeded).  Such a lane's
    difference is the reference's own sensitivity to the last bits of its input (subnormal intermediates,
    cancellation), not a different computation.
      ref_fn(*inputs) -> (c, n) reference outputs; inputs: list of (k_i, n) float32 arrays (directions, xi);
      got: (c, n) GPU outputs of the lanes to prove.
    any_match: also accept a lane where one moved input reproduces every channel within the bar (the test for
    vector-valued outputs such as sampled directions, whose components move together).
    abs_tol: an absolute floor for the bar (unit vectors: 1e-5 of the vector's length)."""
    inputs = [np.asarray(a, np.float32) for a in inputs]
    got = np.asarray(got, np.float64)
    n = got.shape[1]
    if n == 0:
        return np.zeros(0, bool)
    rng = np.random.default_rng(seed)
    moved = []
    for a in inputs:
        st = rng.integers(-k, k + 1, size=(trials,) + a.shape)
        st[0] = 0
        moved.append(np.concatenate([perturb_ulps(a, st[t]) for t in range(trials)], axis=1))
    r = np.asarray(ref_fn(*moved), np.float64).reshape(got.shape[0], trials, n)
    with np.errstate(invalid="ignore"):
        lo = np.nanmin(r, axis=1)
        hi = np.nanmax(r, axis=1)
        tol = np.maximum(REL_TOL * np.maximum(np.maximum(np.abs(lo), np.abs(hi)), FLT_MIN), abs_tol)
        ok = (((got >= lo - tol) & (got <= hi + tol)) | (np.isnan(got) & np.isnan(r).any(axis=1))).all(axis=0)
        if any_match:
            near = np.abs(r - got[:, None, :]) <= np.maximum(REL_TOL * np.maximum(np.abs(r), FLT_MIN), abs_tol)
            ok |= near.all(axis=0).any(axis=0)
    return ok


LIBM_FNS = ["erff", "erfcf", "expf", "logf", "powf", "sinf", "cosf", "tanf", "atanf", "atan2f", "acosf",
            "sincosf(sin)", "sincosf(cos)", "tgammaf"]     # oracle/libm_ulp.c's order


def explained_by_libm_ulp(ref_fn, inputs, got, max_calls=8, any_match=False, abs_tol=0.0):
    """Per-lane proof (libm last bit): True for a lane where the reference itself reproduces the GPU value (every
    channel within the bar) when ONE call of one glibc float function returns its neighbouring float (or all
    calls of it do) -- oracle/libm_ulp.c.  glibc's erff/erfcf are not correctly rounded on ~6 % of inputs, so an
    ill-conditioned output (an inverse-CDF sample at a clamped xi) can hinge on that last bit alone.
      ref_fn(*inputs) -> (c, n): the reference, called here with one lane at a time in this thread (nthreads=1:
      the perturbation switch is per thread)."""
    lib = ref()
    got = np.asarray(got, np.float64)
    n = got.shape[1]
    proven = np.zeros(n, bool)
    if lib is None or n == 0:
        return proven
    nfn = lib.bbmref_libm_nfn()

    def match(r, g):
        with np.errstate(invalid="ignore"):
            tol = np.maximum(REL_TOL * np.maximum(np.abs(r), FLT_MIN), abs_tol)
            return bool(((np.abs(r - g) <= tol) | (r == g) | (np.isnan(r) & np.isnan(g))).all())
    try:
        for i in range(n):
            ins = [np.ascontiguousarray(np.asarray(a, np.float32)[:, i:i + 1]) for a in inputs]
            lib.bbmref_libm_ulp(-1, -1, 0)
            ref_fn(*ins)
            counts = [lib.bbmref_libm_calls(f) for f in range(nfn)]
            for f in range(nfn):
                if proven[i] or counts[f] <= 0:
                    continue
                for call in list(range(min(counts[f], max_calls))) + [-1]:
                    for u in (-1, 1):
                        lib.bbmref_libm_ulp(f, call, u)
                        if match(np.asarray(ref_fn(*ins), np.float64)[:, 0], got[:, i]):
                            proven[i] = True
                            break
                    if proven[i]:
                        break
    finally:
        lib.bbmref_libm_ulp(-1, -1, 0)
    return proven


# ----------------------------------------------------------------- data-driven sampler pdf (He family, Merl)
#
# ndf_sampler's pdf (bbm/ndf_sampler.h:128-156 -> ndf/sampler.h:102-128) is a lookup in a 90-bin CDF built from
# the model's own backscatter evaluations (ndf/sampler.h:143-181, util/cdf.h:39-47).  A CDF entry is a running
# float sum normalised by the total, and a bin's pdf is the difference of two adjacent entries: one ulp in an
# entry near 1 is ~1e-5 of a small bin.  So a 1-ulp difference in a single backscatter evaluation (well inside
# the eval bar) moves the pdf of every direction in the neighbouring bins by up to ~2e-5.  The functions below
# restate that arithmetic in numpy float32 (checked against the reference's own pdf in tests/test_gpu_parity.py)
# so a pdf lane outside the bar can be proven: the GPU value is what the reference's pdf arithmetic gives on the
# CDF built from the GPU's backscatter evaluations, and those evaluations meet the eval bar.

SAMPLER_BINS = 90


def sampler_backscatter_dirs():
    """The 90 halfway vectors h_i at theta = (i/90)^2 pi/2, phi = 0 (ndf/sampler.h:157-166), as (3, 90)."""
    f = np.float32
    q = (np.arange(SAMPLER_BINS, dtype=f) / f(SAMPLER_BINS)).astype(f)
    th = (q.astype(np.float64) ** 2 * np.float64(f(0.5 * np.pi))).astype(f)
    return np.stack([np.sin(th.astype(np.float64)), np.zeros(SAMPLER_BINS),
                     np.cos(th.astype(np.float64))]).astype(f)


def sampler_cdf(backscatter_rgb):
    """util/cdf.h:39-47 over samples hsum(eval(h_i, h_i)) sin(theta1) sqrt(theta1), theta1 = ((i+1)/90)^2 pi/2."""
    f = np.float32
    rgb = np.asarray(backscatter_rgb, f)
    hs = ((f(0) + rgb[0]) + rgb[1]) + rgb[2]
    q1 = (np.arange(1, SAMPLER_BINS + 1, dtype=f) / f(SAMPLER_BINS)).astype(f)
    th1 = (q1.astype(np.float64) ** 2 * np.float64(f(0.5 * np.pi))).astype(f)
    w = (np.sin(th1.astype(np.float64)).astype(f) * np.sqrt(th1)).astype(f)
    acc = np.cumsum((hs * w).astype(f), dtype=f)
    return (acc / acc[-1]).astype(f)


def sampler_pdf(cdf, din, dout):
    """ndf_sampler::pdf(in, out) for component/unit whose CDF is `cdf` (float32 arithmetic as the reference)."""
    f = np.float32
    din = np.asarray(din, f)
    dout = np.asarray(dout, f)
    cdf = np.asarray(cdf, f)
    hx, hy, hz = din[0] + dout[0], din[1] + dout[1], din[2] + dout[2]
    inv = (f(1) / np.sqrt(((f(0) + hx * hx) + hy * hy) + hz * hz)).astype(f)
    h = np.stack([hx * inv, hy * inv, hz * inv]).astype(f)
    sz = np.where(h[2] < 0, f(-1), f(1)).astype(f)
    dz = (h[2] - sz).astype(f)
    nrm = np.sqrt(((f(0) + h[0] * h[0]) + h[1] * h[1]) + dz * dz).astype(f)
    t = 2.0 * np.arcsin(0.5 * nrm.astype(np.float64))
    theta = np.where(h[2] >= 0, t, np.float64(f(np.pi)) - t).astype(f)
    ti = ((np.sqrt(theta / f(0.5 * np.pi)) * f(SAMPLER_BINS)).astype(np.float64) - 0.5).astype(f)
    fl, ce = np.floor(ti), np.ceil(ti)
    w = (ti - fl).astype(f)
    lidx = np.where(fl < 0, SAMPLER_BINS - 1, np.minimum(fl, SAMPLER_BINS - 1)).astype(np.int64)
    uidx = np.where(ce < 0, SAMPLER_BINS - 1, np.minimum(ce, SAMPLER_BINS - 1)).astype(np.int64)
    prev = np.concatenate([[f(0)], cdf[:-1]]).astype(f)
    cp = (cdf - prev).astype(f)
    p = (cp[lidx] * (f(1) - w) + cp[uidx] * w).astype(f)
    st = np.sin(theta.astype(np.float64)).astype(f)
    jac = ((((np.sqrt(theta) * f(f(0.25 * np.pi) * f(np.pi))) / f(SAMPLER_BINS)) * np.abs(st)) * f(2 * np.pi)).astype(f)
    with np.errstate(divide="ignore", invalid="ignore"):
        ph = np.where((h[2] > 0) & (jac > np.finfo(f).eps), p / jac, f(0)).astype(f)
        oh = ((f(0) + dout[0] * h[0]) + dout[1] * h[1]) + dout[2] * h[2]
        pdf = (ph.astype(np.float64) / np.abs(4.0 * oh.astype(np.float64))).astype(f)
    return np.where((dout[2] > 0) & (din[2] > 0), pdf, f(0))


def max_rel_normal(got, ref):
    """max |gpu - ref| / |ref| over the lanes with a normal (|ref| >= FLT_MIN) finite reference value."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    sel = np.isfinite(ref) & (np.abs(ref) >= FLT_MIN)
    if not sel.any():
        return 0.0
    with np.errstate(invalid="ignore"):
        r = np.abs(got[sel] - ref[sel]) / np.abs(ref[sel])
    r[np.isnan(r)] = np.inf
    return float(r.max())


# ------------------------------------------------------------------------------ directions

def dirgen_numpy(seed, stream_id, offset, n, mode=0):
    """numpy restatement of bbm_hip_fill_directions' counter formula (float64 trig): used to
    check that shards regenerate disjoint slices of one global batch."""
    m64 = (1 << 64) - 1

    def mix64(z):
        z = np.asarray(z, dtype=np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        return z ^ (z >> np.uint64(31))

    with np.errstate(over="ignore"):
        key = int(mix64(np.uint64(seed & m64))) ^ ((0xd1b54a32d192ed03 * (stream_id + 1)) & m64)
        idx = np.arange(offset, offset + n, dtype=np.uint64)
        h = mix64(np.uint64(key) + np.uint64(0x9e3779b97f4a7c15) * idx)
    u1 = (h >> np.uint64(40)).astype(np.float64) / 16777216.0
    u2 = ((h >> np.uint64(16)) & np.uint64(0xffffff)).astype(np.float64) / 16777216.0
    z = u1 if mode == 0 else 2.0 * u1 - 1.0
    s = np.sqrt(np.maximum(1.0 - z * z, 0.0))
    phi = 2.0 * np.pi * u2
    return np.stack([s * np.cos(phi), s * np.sin(phi), z]).astype(np.float32)


# ------------------------------------------------------------------------------ fitting

def golden_fit():
    with open(os.path.join(GOLDEN, "fit.json")) as f:
        meta = json.load(f)
    return meta, np.load(os.path.join(GOLDEN, "fit.npz"))


def _grid_desc(g):
    s_in = np.asarray(g["samples_in"], np.uint64)
    s_out = np.asarray(g["samples_out"], np.uint64)
    rng = np.asarray(list(g["start_in"]) + list(g["end_in"]) + list(g["start_out"]) + list(g["end_out"]), np.float32)
    return s_in, s_out, rng


def ref_loss_total(name, fitted, reference, grid, loss_kind):
    """The reference's own sampledlossfunction()() total (serial float sum / N) on a spherical grid."""
    lib = ref()
    s_in, s_out, rng = _grid_desc(grid)
    fitted = np.ascontiguousarray(fitted, np.float32)
    reference = np.ascontiguousarray(reference, np.float32)
    tot = np.zeros(1, np.float32)
    n = lib.bbmref_loss(name.encode(), _fp(fitted), _fp(reference), fitted.size, 0, _fp(s_in), _fp(s_out), _fp(rng),
                        loss_kind, None, _fp(tot), 1)
    assert n > 0
    return np.float32(tot[0])


def ref_pair_losses(name, fitted, reference, din, dout, loss_kind, nthreads=8, lib=None):
    """Per-sample reference losses on explicit direction pairs (the reference's sampledlossfunction
    over a table linearizer, oracle/ref_fit.cpp): (n,) float32."""
    lib = lib or ref()
    din = np.ascontiguousarray(din, np.float32)
    dout = np.ascontiguousarray(dout, np.float32)
    n = din.shape[1]
    ptrs = (ctypes.c_void_p * 6)(*[din[k].ctypes.data for k in range(3)] + [dout[k].ctypes.data for k in range(3)])
    s_in = np.asarray([n, 0], np.uint64)
    fitted = np.ascontiguousarray(fitted, np.float32)
    reference = np.ascontiguousarray(reference, np.float32)
    per = np.zeros(n, np.float32)
    rc = lib.bbmref_loss(name.encode(), _fp(fitted), _fp(reference), fitted.size, 2, _fp(s_in), _fp(s_in),
                         ctypes.cast(ptrs, ctypes.c_void_p), loss_kind, _fp(per), None, nthreads)
    assert rc == n, rc
    return per


def ref_batch_indices(seed, nsamples, batchsize, updates):
    """The indices the reference's bbm::batch draws (bbm::rng<Size_t>, batch.h:40-54) after construction and after
    each of `updates` update() calls -> (updates + 1, batchsize) uint64 (oracle/ref_fit.cpp: bbmref_batch_indices)."""
    lib = ref()
    out = np.zeros((updates + 1, batchsize), np.uint64)
    rc = lib.bbmref_batch_indices(ctypes.c_uint64(seed), ctypes.c_uint64(nsamples), ctypes.c_size_t(batchsize),
                                  ctypes.c_int(updates), _fp(out))
    assert rc == 0, rc
    return out


def ref_batch_losses(name, fitted, reference, grid, loss_kind, seed, batchsize, updates):
    """batch::operator()(idx) of the reference's bbm::batch over its sampledlossfunction on a spherical grid, for
    idx in [0, batchsize) after construction and after each update() -> (updates + 1, batchsize) float32."""
    lib = ref()
    s_in, s_out, rng = _grid_desc(grid)
    fitted = np.ascontiguousarray(fitted, np.float32)
    reference = np.ascontiguousarray(reference, np.float32)
    out = np.zeros((updates + 1, batchsize), np.float32)
    rc = lib.bbmref_batch_loss(name.encode(), _fp(fitted), _fp(reference), fitted.size, 0, _fp(s_in), _fp(s_out),
                               _fp(rng), loss_kind, ctypes.c_uint64(seed), ctypes.c_size_t(batchsize),
                               ctypes.c_int(updates), _fp(out))
    assert rc > 0, rc
    return out


def golden_batch():
    with open(os.path.join(GOLDEN, "batch.json")) as f:
        return json.load(f)


def ref_merl_index(din, dout, h=(1, 90), d=(180, 90)):
    """The reference merl_linearizer's inverse map (direction pair -> index)."""
    lib = ref()
    din = np.ascontiguousarray(din, np.float32)
    dout = np.ascontiguousarray(dout, np.float32)
    n = din.shape[1]
    idx = np.zeros(n, np.uint64)
    sh = np.asarray(h, np.uint64)
    sd = np.asarray(d, np.uint64)
    lib.bbmref_merl_index(_fp(sh), _fp(sd), ctypes.c_size_t(n), _fp(din[0]), _fp(din[1]), _fp(din[2]), _fp(dout[0]),
                          _fp(dout[1]), _fp(dout[2]), _fp(idx))
    return idx


class RefTotalLoss:
    """A SampledLoss stand-in scored by the reference itself (serial float totals): drives the host
    compass logic of bbm_amd.fit.Compass on the CPU with exactly the reference's loss values."""

    def __init__(self, fitted, reference_params, grid, loss_kind):
        self.fitted = fitted
        self.reference = np.asarray(reference_params, np.float32)
        self.grid = grid
        self.loss_kind = loss_kind
        self.calls = 0

    def update(self):
        """concepts::lossfunction's update() (sampledlossfunction.h:52: nothing to do)."""

    def probe_losses(self, probes):
        self.calls += 1
        return np.array([ref_loss_total(self.fitted.name, p, self.reference, self.grid, self.loss_kind)
                         for p in np.asarray(probes, np.float32)], np.float32)

    def __call__(self, params=None):
        p = self.fitted._params if params is None else params
        return float(self.probe_losses(np.asarray(p, np.float32)[None])[0])


def merl_directions_f64(h=(1, 90), d=(180, 90)):
    """merl_linearizer's index -> direction map (include/linearizer/merl_linearizer.h:49-83) evaluated in
    float64 (numpy): the sample at index i sits on the lower edge of its (theta_h, theta_d, phi_d) bin;
    convertFromHalfwayDifference (include/core/vec_transform.h:118-123) = rotZ(phi_h) rotY(theta_h)."""
    n = d[0] * d[1] * h[1]
    i = np.arange(n, dtype=np.int64)
    pd = i % d[0]
    td = (i // d[0]) % d[1]
    th = i // (d[0] * d[1])
    theta_h = (th / h[1]) ** 2 * (0.5 * np.pi)
    phi_d = pd / d[0] * np.pi
    theta_d = td / d[1] * (0.5 * np.pi)
    diff = np.stack([np.cos(phi_d) * np.sin(theta_d), np.sin(phi_d) * np.sin(theta_d), np.cos(theta_d)])
    cy, sy = np.cos(theta_h), np.sin(theta_h)

    def rot(v):      # phi_h == 0: rotZ is the identity
        return np.stack([cy * v[0] + sy * v[2], v[1], -sy * v[0] + cy * v[2]])

    din = rot(diff)
    dout = rot(np.stack([-diff[0], -diff[1], diff[2]]))
    din[2] = np.maximum(din[2], 0)
    dout[2] = np.maximum(dout[2], 0)
    return din, dout


# ------------------------------------------------------------------------------------------ Merl

def synthetic_merl(path, seed=20240611):
    """Write a synthetic MERL-MIT .binary (no measured data ships with the reference): a smooth
    specular-plus-diffuse table over (theta_h, theta_d, phi_d) with noise, and 2 % of the entries set to
    -1 as in the measured files' unmeasured bins (merl.h:200-202 clamps them to 0).  Returns the raw
    (3, 90, 90, 180) float64 array."""
    from bbm_amd.merl import write_binary
    rng = np.random.default_rng(seed)
    th, td, pd = np.meshgrid(np.arange(90) / 90.0, np.arange(90) / 90.0, np.arange(180) / 180.0, indexing="ij")
    rgb = np.empty((3, 90, 90, 180))
    for c, (a, b) in enumerate(((900.0, 60.0), (700.0, 90.0), (400.0, 120.0))):
        rgb[c] = a * np.exp(-8.0 * th * th) * (1 + 0.5 * np.cos(2 * np.pi * pd)) + b * (1 + td) \
            + rng.normal(0.0, 5.0, th.shape)
    rgb[rng.random(rgb.shape) < 0.02] = -1.0
    write_binary(path, rgb)
    return rgb


def merl_table_numpy(raw):
    """merl_data::import's white balance (merl.h:199-203) in float64, rounded to float as lookup<Spectrum>
    does: (3, 90*90*180) float32."""
    raw = raw.reshape(3, -1)
    w = (1.0, 1.15, 1.66)
    return np.stack([np.fmax(0.0, raw[c] * w[c] / 1500.0) for c in range(3)]).astype(np.float32)


def ref_merl_eval_pdf(filename, din, dout, component=3, unit=0, nthreads=8):
    lib = ref()
    din = np.ascontiguousarray(din, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    n = din.shape[1]
    res = np.zeros((4, n), np.float32)
    rc = lib.bbmref_merl_eval_pdf(str(filename).encode(), ctypes.c_size_t(n), _fp(din[0]), _fp(din[1]), _fp(din[2]),
                                  _fp(dout[0]), _fp(dout[1]), _fp(dout[2]), ctypes.c_uint32(component),
                                  ctypes.c_uint32(unit), 3, _fp(res[0]), _fp(res[1]), _fp(res[2]), _fp(res[3]),
                                  nthreads)
    if rc != 0:
        raise RuntimeError(f"reference rejected MERL file {filename}")
    return res


def ref_merl_sample(filename, dout, xi, component=3, unit=0):
    lib = ref()
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    xi = np.ascontiguousarray(xi, dtype=np.float32)
    n = dout.shape[1]
    d = np.zeros((4, n), np.float32)
    flag = np.zeros(n, np.uint32)
    rc = lib.bbmref_merl_sample(str(filename).encode(), ctypes.c_size_t(n), _fp(dout[0]), _fp(dout[1]), _fp(dout[2]),
                                _fp(xi[0]), _fp(xi[1]), ctypes.c_uint32(component), ctypes.c_uint32(unit),
                                _fp(d[0]), _fp(d[1]), _fp(d[2]), _fp(d[3]), _fp(flag))
    if rc != 0:
        raise RuntimeError(f"reference rejected MERL file {filename}")
    return d, flag


def ref_merl_to_string(filename):
    lib = ref()
    buf = ctypes.create_string_buffer(4096)
    if lib.bbmref_merl_to_string(str(filename).encode(), buf, 4096) < 0:
        raise RuntimeError(f"reference rejected MERL file {filename}")
    return buf.value.decode()


# ------------------------------------------------------------------ runtime aggregates (oracle/ref_runtime.cpp)

def runtime_tree(tree):
    """Preorder arrays of a runtime-aggregate tree: `tree` is (name, params) for a model or ("Aggregate", [kids])."""
    names, nkids, nps, params = [], [], [], []

    def walk(t):
        if t[0] == "Aggregate":
            names.append(b"Aggregate")
            nkids.append(len(t[1]))
            nps.append(0)
            for k in t[1]:
                walk(k)
        else:
            p = np.asarray(t[1], np.float32).reshape(-1)
            names.append(t[0].encode())
            nkids.append(0)
            nps.append(p.size)
            params.append(p)
    walk(tree)
    arr = (ctypes.c_char_p * len(names))(*names)
    return (len(names), arr, (ctypes.c_int * len(nkids))(*nkids),
            np.ascontiguousarray(np.concatenate(params) if params else np.zeros(0), np.float32),
            (ctypes.c_int * len(nps))(*nps))


def ref_runtime_eval_pdf(tree, din, dout, component=3, unit=0, nthreads=8, f64=False):
    """(4, N): eval RGB + pdf of the reference's runtime aggregate (aggregatebsdf of bsdf_ptrs, what
    fromString<bsdf_ptr> builds), floatRGB (float32 directions) or doubleRGB (f64: float64 directions)."""
    lib = ref()
    k, names, nk, params, nps = runtime_tree(tree)
    dt = np.float64 if f64 else np.float32
    din = np.ascontiguousarray(din, dtype=dt)
    dout = np.ascontiguousarray(dout, dtype=dt)
    n = din.shape[1]
    res = np.zeros((4, n), dt)
    fn = lib.bbmref_runtime_eval_pdf_dd if f64 else lib.bbmref_runtime_eval_pdf
    rc = fn(k, names, nk, _fp(params), nps, ctypes.c_size_t(n), _fp(din[0]), _fp(din[1]), _fp(din[2]), _fp(dout[0]),
            _fp(dout[1]), _fp(dout[2]), ctypes.c_uint32(component), ctypes.c_uint32(unit), 3, _fp(res[0]), _fp(res[1]),
            _fp(res[2]), _fp(res[3]), nthreads)
    if rc != 0:
        raise KeyError(f"oracle cannot build the runtime aggregate {tree!r}")
    return res


def ref_runtime_sample(tree, dout, xi, component=3, unit=0, nthreads=8, f64=False):
    """((4, N) direction + pdf, (N,) flags) of the reference's runtime aggregate's sample."""
    lib = ref()
    k, names, nk, params, nps = runtime_tree(tree)
    dt = np.float64 if f64 else np.float32
    dout = np.ascontiguousarray(dout, dtype=dt)
    xi = np.ascontiguousarray(xi, dtype=dt)
    n = dout.shape[1]
    res = np.zeros((4, n), dt)
    flag = np.zeros(n, np.uint32)
    fn = lib.bbmref_runtime_sample_dd if f64 else lib.bbmref_runtime_sample
    rc = fn(k, names, nk, _fp(params), nps, ctypes.c_size_t(n), _fp(dout[0]), _fp(dout[1]), _fp(dout[2]), _fp(xi[0]),
            _fp(xi[1]), ctypes.c_uint32(component), ctypes.c_uint32(unit), _fp(res[0]), _fp(res[1]), _fp(res[2]),
            _fp(res[3]), flag.ctypes.data_as(ctypes.c_void_p), nthreads)
    if rc != 0:
        raise KeyError(f"oracle cannot build the runtime aggregate {tree!r}")
    return res, flag


def ref_runtime_reflectance(tree, dout, component=3, unit=0, f64=False):
    lib = ref()
    k, names, nk, params, nps = runtime_tree(tree)
    dt = np.float64 if f64 else np.float32
    dout = np.ascontiguousarray(dout, dtype=dt)
    n = dout.shape[1]
    res = np.zeros((3, n), dt)
    fn = lib.bbmref_runtime_reflectance_dd if f64 else lib.bbmref_runtime_reflectance
    rc = fn(k, names, nk, _fp(params), nps, ctypes.c_size_t(n), _fp(dout[0]), _fp(dout[1]), _fp(dout[2]),
            ctypes.c_uint32(component), ctypes.c_uint32(unit), _fp(res[0]), _fp(res[1]), _fp(res[2]))
    if rc != 0:
        raise KeyError(f"oracle cannot build the runtime aggregate {tree!r}")
    return res


def runtime_fit_tree(key, params):
    """The runtime-aggregate tree (runtime_tree) of a fused key "Aggregate<A,B>" at its flat parameter vector: what
    bsdf_import builds from the material's fits/ line."""
    names = key[len("Aggregate<"):-1].split(",")
    p = np.asarray(params, np.float32)
    kids, k = [], 0
    for nm in names:
        m = len(ref_default_params(nm))
        kids.append((nm, p[k:k + m]))
        k += m
    assert k == p.size, (key, p.size)
    return ("Aggregate", kids)
