"""bbm_amd -- an MI355X-native (gfx950) batched BSDF backbone for bsdfbenchmark/bbm.

The hot path of BBM -- bsdfmodel<>::eval / pdf / sample over many (in, out) direction pairs --
runs in libbbm_hip.so (hand-written HIP kernels, C-ABI in include/bbm_hip.h).  This package is
the host-side mirror of the reference's model interface: one constructor per exported model
name, `fromString` / `bsdf_import`, `bsdf_flag`, `unit_t`, `BsdfSample`, and batched
`eval` / `pdf` / `eval_pdf` / `sample` on torch CUDA tensors.

Importing the package loads the HIP library; if it is missing the import fails loudly.
"""
from . import _lib
from .backbone import (Aggregate, AggregateModel, BsdfModel, BsdfSample, bsdf_flag, bsdf_import, fill_directions, fromString,
                       parse_model, model_names, scratch_bytes, scratch_trim, scratch_trim_captured, set_exact_subnormals, unit_t, _make_ctor)
from .models import ATTRIBUTES

_lib.load()

__all__ = ["Aggregate", "AggregateModel", "BsdfModel", "BsdfSample", "bsdf_flag", "unit_t", "fromString", "bsdf_import",
           "parse_model", "model_names",
           "fill_directions", "scratch_trim", "scratch_trim_captured", "scratch_bytes", "set_exact_subnormals", "ATTRIBUTES"]

from .merl import Merl  # noqa: E402  -- measured data: constructed from a file, not from attributes

__all__.append("Merl")

for _name in model_names():
    if _name.isidentifier() and _name != "Merl":          # Aggregate<Lambertian,X> entries are built with Aggregate(...)
        globals()[_name] = _make_ctor(_name)
        __all__.append(_name)
del _name
