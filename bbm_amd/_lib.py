"""ctypes binding of libbbm_hip.so (C-ABI: include/bbm_hip.h).

The library is built in-tree by __graft_entry__.build() (hipcc --offload-arch=gfx950) into
bbm_amd/lib/libbbm_hip.so.  There is no fallback: if the library is missing or fails to load,
every entry point raises, so a GPU run can never silently take a CPU path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BBM_HIP_LIB") or os.path.join(_HERE, "lib", "libbbm_hip.so")

# return codes (include/bbm_hip.h)
OK = 0
ERR_INVALID_MODEL = -1
ERR_INVALID_ARG = -2
ERR_UNSUPPORTED = -3
ERR_HIP = -4

# exported symbols and their signatures: (restype, argtypes)
_P = ctypes.c_void_p
_F = ctypes.c_float
_I = ctypes.c_int
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t

SIGNATURES = {
    "bbm_hip_abi_version": (_I, []),
    "bbm_hip_set_exact_subnormals": (_I, [_I]),
    "bbm_hip_last_error": (ctypes.c_char_p, []),
    "bbm_hip_num_models": (_I, []),
    "bbm_hip_model_name": (ctypes.c_char_p, [_I]),
    "bbm_hip_model_id": (_I, [ctypes.c_char_p]),
    "bbm_hip_model_nparams": (_I, [_I]),
    "bbm_hip_model_params": (_I, [_I, _I, _P, _I]),
    "bbm_hip_model_components": (_I, [_I]),
    "bbm_hip_eval": (_I, [_I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P]),
    "bbm_hip_pdf": (_I, [_I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P]),
    "bbm_hip_eval_pdf": (_I, [_I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P]),
    "bbm_hip_sample": (_I, [_I, _P, _I, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P, _P]),
    "bbm_hip_reflectance": (_I, [_I, _P, _I, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P]),
    "bbm_hip_model_has_f64": (_I, [_I]),
    "bbm_hip_eval_pdf_f64": (_I, [_I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P]),
    "bbm_hip_sample_f64": (_I, [_I, _P, _I, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P, _P]),
    "bbm_hip_reflectance_f64": (_I, [_I, _P, _I, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P]),
    "bbm_hip_fill_directions": (_I, [_U64, _U32, _U64, _SZ, _I, _P, _P, _P, _P]),
    "bbm_hip_model_param_attrs": (_I, [_I, _P, _I]),
    "bbm_hip_linearizer_size": (_I, [_P, _P]),
    "bbm_hip_linearize": (_I, [_P, _U64, _SZ, _P, _P, _P, _P, _P, _P, _P]),
    "bbm_hip_loss_workspace_size": (_SZ, [_I]),
    "bbm_hip_loss": (_I, [_I, _P, _I, _I, _P, _U64, _SZ, _P, _P, _P, _I, _U32, _U32, _P, _P, _SZ, _P]),
    "bbm_hip_loss_pairs": (_I, [_I, _P, _I, _I, _SZ, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _U32, _U32, _P, _P, _SZ,
                                _P]),
    "bbm_hip_epd_g1_table": (_I, [_P, _I]),
    "bbm_hip_merl_table": (_I, [_P, _U32, _U32, _U32, _P, _P]),
    "bbm_hip_check_workspace_size": (_SZ, [_P]),
    "bbm_hip_check": (_I, [_I, _P, _I, _P, _P, _P, _P, _SZ, _P]),
    "bbm_hip_check_draws": (_I, [_I, _U64, _I, _I, _U64, _SZ, _P, _P, _P]),
    "bbm_hip_check_trials": (_I, [_I, _U64, _I, _I, _P, _P, _P, _P]),
    "bbm_hip_sphere_dirs": (_I, [_P, _P, _SZ, _I, _P, _P, _P, _P]),
    "bbm_hip_aggregate_eval_pdf": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P]),
    "bbm_hip_aggregate_sample": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P, _P]),
    "bbm_hip_aggregate_reflectance": (_I, [_P, _I, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P]),
    "bbm_hip_model_layout": (ctypes.c_char_p, [_I]),
    "bbm_hip_parse_model": (_I, [ctypes.c_char_p, _P, _P, _P, _I, _I]),
    "bbm_hip_parse_model_tree": (_I, [ctypes.c_char_p, _P, _P, _P, _P, _I, _I]),
    "bbm_hip_aggregate_eval_pdf_f64": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P]),
    "bbm_hip_aggregate_sample_f64": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P, _P, _P]),
    "bbm_hip_aggregate_reflectance_f64": (_I, [_P, _I, _P, _P, _P, _P, _SZ, _U32, _U32, _P, _P, _P, _P]),
    "bbm_hip_scratch_trim": (_SZ, []),
    "bbm_hip_scratch_trim_captured": (_SZ, []),
    "bbm_hip_scratch_bytes": (_SZ, []),
    "bbm_hip_libm_eval": (_I, [_I, _P, _P, _P, _SZ, _P]),
    "bbm_hip_loss_tree_workspace_size": (_SZ, [_I, _SZ]),
    "bbm_hip_loss_tree": (_I, [_P, _I, _P, _I, _I, _SZ, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _U32, _U32, _P, _P, _SZ,
                               _P]),
    "bbm_hip_loss_tree_f64": (_I, [_P, _I, _P, _I, _I, _SZ, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _U32, _U32, _P, _P,
                                   _SZ, _P]),
    "bbm_hip_check_tree_workspace_size": (_SZ, [_P]),
    "bbm_hip_check_tree": (_I, [_P, _I, _P, _P, _P, _P, _SZ, _P]),
    "bbm_hip_check_tree_f64": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "bbm_hip_rng_init": (_I, [_P, _U64, _U64, _U64]),
    "bbm_hip_rng_draw": (_I, [_P, _P, _SZ]),
    "bbm_hip_gather_samples": (_I, [_P, _SZ, _U64, _P, _P, _I, _P]),
    "bbm_hip_gather_samples_f64": (_I, [_P, _SZ, _U64, _P, _P, _I, _P]),
    "bbm_hip_comm_unique_id": (_I, [_P, _SZ]),
    "bbm_hip_comm_init": (_I, [_P, _SZ, _I, _I, _P]),
    "bbm_hip_comm_destroy": (_I, [_P]),
    "bbm_hip_comm_rank": (_I, [_P]),
    "bbm_hip_comm_size": (_I, [_P]),
    "bbm_hip_allreduce_sums": (_I, [_P, _P, _SZ, _P]),
}

ABI_VERSION = 12
CALL_EXACT = 0x20000000     # BBM_HIP_CALL_EXACT: OR-ed into a model id, this call in exact mode
CALL_DEFAULT = 0x10000000   # BBM_HIP_CALL_DEFAULT: this call in default mode (whatever set_exact_subnormals says)
AGGREGATE = -100        # BBM_HIP_AGGREGATE: model id of a composed-aggregate node (bbm_hip_child.children)
AGGREGATE_BSDF = -101   # BBM_HIP_AGGREGATE_BSDF: a composed runtime aggregate (aggregatebsdf, what fromString builds)
RUNTIME_AGGREGATE = 0x40000000   # BBM_HIP_RUNTIME_AGGREGATE: OR-ed into a fused aggregate's id -> aggregatebsdf semantics


class Child(ctypes.Structure):
    """bbm_hip_child (include/bbm_hip.h): one child of a composed aggregate -- a registry model with its float
    parameters, or (model_id = AGGREGATE) a nested composed aggregate with its own children."""
    _fields_ = [("model_id", ctypes.c_int), ("params", ctypes.c_void_p), ("nparams", ctypes.c_int),
                ("children", ctypes.c_void_p), ("nchildren", ctypes.c_int)]


class ChildF64(ctypes.Structure):
    """bbm_hip_child_f64: the same with double parameters (doubleRGB)."""
    _fields_ = [("model_id", ctypes.c_int), ("params", ctypes.c_void_p), ("nparams", ctypes.c_int),
                ("children", ctypes.c_void_p), ("nchildren", ctypes.c_int)]


class Rng(ctypes.Structure):
    """bbm_hip_rng (include/bbm_hip.h): the state of bbm::rng<Size_t> (std::mt19937_64 + uniform_int_distribution)."""
    _fields_ = [("mt", ctypes.c_uint64 * 312), ("pos", ctypes.c_uint64), ("lower", ctypes.c_uint64),
                ("upper", ctypes.c_uint64), ("magic", ctypes.c_uint64)]


COMM_ID_BYTES = 128     # BBM_HIP_COMM_ID_BYTES
RNG_DEFAULT_SEED = 5489  # BBM_HIP_RNG_DEFAULT_SEED (std::mt19937_64::default_seed)


class BackboneError(RuntimeError):
    """Raised when a libbbm_hip call fails (the reference throws std::runtime_error /
    std::invalid_argument, include/core/error.h:42-46)."""

    def __init__(self, code, message):
        super().__init__(f"libbbm_hip error {code}: {message}")
        self.code = code


_lib = None


def load():
    """Load (once) and return the ctypes handle; raises if the HIP library is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    if not hasattr(lib, "bbm_hip_abi_version") or lib.bbm_hip_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI {lib.bbm_hip_abi_version() if hasattr(lib, 'bbm_hip_abi_version') else '?'}, "
                          f"this package needs ABI {ABI_VERSION}: rebuild it")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(code):
    """Turn a negative return code into BackboneError with the library's message."""
    if code < 0:
        msg = load().bbm_hip_last_error()
        raise BackboneError(code, msg.decode() if msg else "")
    return code
