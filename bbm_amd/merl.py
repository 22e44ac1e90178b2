"""Merl: the MERL-MIT measured BRDF (include/staticmodel/merl.h) as a batched GPU model.

The reference's `merl<CONF>` is `ndf_sampler<merl_data<CONF, "Merl">, 90, 1>` (merl.h:224-225): eval
looks the (theta_h, theta_d, phi_d) bin of (in, out) up in the 90 x 90 x 180 table read from a MERL
.binary file (three uint32 dimensions, then the R, G and B planes as doubles), white-balanced on import
(merl.h:173-206); sample / pdf are the data-driven backscatter sampler; reflectance is a placeholder.

Here the file is read on the host, its doubles are copied to the GPU once and turned into the model's
float4 table there (bbm_hip_merl_table); the model's two parameters are the table's device address, so
a `Merl` evaluates through the same C-ABI entry points as every other model.  The table (23 MB) lives
as long as the object.
"""
import ctypes

import numpy as np

from . import _lib
from .backbone import BsdfModel, _stream_ptr, _torch

DIMS = (90, 90, 180)        # theta_h, theta_d, phi_d (merl.h:184)


def read_binary(filename):
    """(dims, raw) of a MERL-MIT .binary file; raw = the 3 x prod(dims) doubles (R, G, B planes).
    Errors follow merl_data::import (merl.h:176-184)."""
    try:
        with open(filename, "rb") as f:
            dims = np.fromfile(f, dtype="<u4", count=3)
            if dims.size != 3 or tuple(int(d) for d in dims) != DIMS:
                raise RuntimeError(f"BBM: not a recognized MERL BRDF: \"{filename}\"")
            size = 3 * int(np.prod(dims, dtype=np.int64))
            raw = np.fromfile(f, dtype="<f8", count=size)
    except OSError:
        raise RuntimeError(f"BBM: unable to open MERL BRDF: \"{filename}\"") from None
    if raw.size != size:
        raise RuntimeError(f"BBM: truncated MERL BRDF: \"{filename}\" ({raw.size} of {size} values)")
    return tuple(int(d) for d in dims), raw


def write_binary(filename, rgb):
    """Write a (3, 90, 90, 180) array (R, G, B planes indexed [theta_h, theta_d, phi_d]) as a MERL .binary."""
    rgb = np.ascontiguousarray(rgb, dtype="<f8")
    if rgb.shape != (3,) + DIMS:
        raise ValueError(f"expected a (3, 90, 90, 180) array, got {rgb.shape}")
    with open(filename, "wb") as f:
        np.asarray(DIMS, dtype="<u4").tofile(f)
        rgb.tofile(f)


WHITE_BALANCE = (1.0, 1.15, 1.66)   # merl.h:200-202: channel c of the table is max(0, raw_c * w_c / 1500)


def encode(rgb):
    """Inverse of the import's white balance: a (3, 90*90*180) table of BRDF values (e.g. an analytic
    model evaluated at the merl_linearizer bin centres) -> the (3, 90, 90, 180) raw doubles a MERL
    .binary holds."""
    rgb = np.asarray(rgb, dtype=np.float64).reshape(3, -1)
    return np.stack([rgb[c] * 1500.0 / WHITE_BALANCE[c] for c in range(3)]).reshape((3,) + DIMS)


class Merl(BsdfModel):
    """Merl(filename) -- bbm::merl<floatRGB> (staticmodel/merl.h:224-225) on the current CUDA device."""

    def __init__(self, filename, *, stream=None):
        torch = _torch()
        lib = _lib.load()
        dims, raw = read_binary(filename)
        mid = lib.bbm_hip_model_id(b"Merl")
        if mid < 0:
            raise _lib.BackboneError(mid, "model Merl is not available in libbbm_hip")
        dev = torch.device("cuda", torch.cuda.current_device())
        raw_dev = torch.from_numpy(raw).to(dev)
        self.table = torch.empty((int(np.prod(dims)), 4), dtype=torch.float32, device=dev)
        _lib.check(lib.bbm_hip_merl_table(ctypes.c_void_p(raw_dev.data_ptr()), dims[0], dims[1], dims[2],
                                          ctypes.c_void_p(self.table.data_ptr()), _stream_ptr(stream)))
        (torch.cuda.current_stream() if stream is None else stream).synchronize()   # raw_dev is freed next
        del raw_dev
        self.name = "Merl"
        self.model_id = mid
        self.filename = str(filename)
        ptr = self.table.data_ptr()
        self._params = np.array([ptr & 0xFFFFFFFF, ptr >> 32], dtype=np.uint32).view(np.float32)

    def _pptr(self):
        # the parameters are the table's device address: valid only on the device that holds it (and only while
        # this object, which owns the table, is alive -- the C-ABI and C++ callers' contract as well)
        torch = _torch()
        if torch.cuda.current_device() != self.table.device.index:
            raise RuntimeError(f"Merl table lives on cuda:{self.table.device.index}, current device is "
                               f"cuda:{torch.cuda.current_device()}")
        return super()._pptr()

    def set_parameter_values(self, values):
        raise TypeError("Merl has no settable parameters (measured data)")

    def parameter_values(self, flag=None):
        return np.zeros(0, np.float32) if flag is not None else self._params.copy()

    def __str__(self):
        # merl_data::toString (merl.h:161-164) with the quoted string conversion (core/stringconvert.h:247-250)
        return f"Merl(\"{self.filename}\")"

    __repr__ = __str__
