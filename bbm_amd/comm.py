"""RCCL communicator of the C-ABI (bbm_hip_comm_*, bbm_hip_allreduce_sums): the loss reduction of a fit sharded over
the GPUs of a node without torch.distributed -- what a C++ caller of the library uses (backbone/hip/include/bbm_hip/
fit.h).  One process per GPU; rank 0 makes the id (`unique_id()`), every rank builds `Comm(id, rank, world)` on its
current device, and `allreduce_sums(t)` sums a float64 CUDA tensor in place over the ranks (ncclSum, ncclFloat64)."""
import ctypes

from . import _lib
from .backbone import _stream_ptr


def unique_id():
    """ncclGetUniqueId -> bytes (BBM_HIP_COMM_ID_BYTES); rank 0 makes it and hands it to the others."""
    buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    _lib.check(_lib.load().bbm_hip_comm_unique_id(buf, _lib.COMM_ID_BYTES))
    return bytes(buf)


class Comm:
    """bbm_hip_comm: an RCCL communicator over `world` ranks, this process being `rank` (its current HIP device)."""

    def __init__(self, uid, rank, world):
        uid = bytes(uid)
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError(f"unique id must be {_lib.COMM_ID_BYTES} bytes")
        self._h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * len(uid)).from_buffer_copy(uid)
        _lib.check(_lib.load().bbm_hip_comm_init(buf, len(uid), int(rank), int(world), ctypes.byref(self._h)))

    @property
    def rank(self):
        return _lib.check(_lib.load().bbm_hip_comm_rank(self._h))

    @property
    def size(self):
        return _lib.check(_lib.load().bbm_hip_comm_size(self._h))

    def allreduce_sums(self, sums, stream=None):
        """In-place sum over the ranks of a contiguous float64 CUDA tensor (stream-ordered on `stream`)."""
        if sums.dtype.itemsize != 8 or not sums.is_contiguous():
            raise ValueError("allreduce_sums takes a contiguous float64 tensor")
        _lib.check(_lib.load().bbm_hip_allreduce_sums(self._h, sums.data_ptr(), sums.numel(), _stream_ptr(stream)))
        return sums

    def close(self):
        if self._h:
            _lib.check(_lib.load().bbm_hip_comm_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
