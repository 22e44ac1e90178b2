"""bbm::batch's index generator and the RCCL / gather plumbing of the C-ABI, on the CPU (no kernel runs):

* bbm_hip_rng (std::mt19937_64 + libstdc++'s uniform_int_distribution, backbone/native/include/backbone/random.h:40-66)
  draws exactly the indices the reference's bbm::batch draws (include/bbm/batch.h:40-54) -- pinned by
  tests/golden/batch.json (oracle/gen_batch_golden.py, the reference's own batch) and, where the reference shim is
  built, by the reference live for more seeds and sample counts;
* the Python mirror (bbm_amd.fit.Batch / BatchRng) follows the reference's construction order (one draw in the
  constructor, one per update());
* argument validation of the gather and communicator entry points fails before any device call.
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_util as ou

GOLDEN = ou.golden_batch()


@pytest.fixture(scope="module")
def lib():
    from bbm_amd import _lib
    return _lib.load()


@pytest.mark.parametrize("case", range(len(GOLDEN["indices"])))
def test_rng_draws_the_references_batch_indices(case):
    from bbm_amd import fit
    g = GOLDEN["indices"][case]
    rng = fit.BatchRng(g["seed"], 0, g["samples"])
    got = np.concatenate([rng.draw(g["batchsize"]) for _ in range(g["updates"] + 1)])
    np.testing.assert_array_equal(got, np.asarray(g["index"], np.uint64))
    assert got.max() <= g["samples"]


@pytest.mark.skipif(ou.ref() is None, reason="reference shim not built")
@pytest.mark.parametrize("seed", [0, 42, 2 ** 63 + 5])
@pytest.mark.parametrize("n", [1, 2, 1000, 4_000_000])
def test_rng_against_live_reference(seed, n):
    from bbm_amd import fit
    want = ou.ref_batch_indices(seed, n, 200, 2)
    rng = fit.BatchRng(seed, 0, n)
    got = np.stack([rng.draw(200) for _ in range(3)])
    np.testing.assert_array_equal(got, want)


def test_rng_bounds_and_validation(lib):
    from bbm_amd import _lib, fit
    r = fit.BatchRng(7, 10, 12)
    v = r.draw(10000)
    assert v.min() == 10 and v.max() == 12
    assert set(np.unique(v)) == {10, 11, 12}
    full = fit.BatchRng(7).draw(4)                       # [0, 2^64 - 1]: the generator's own output
    assert full.dtype == np.uint64
    st = _lib.Rng()
    assert lib.bbm_hip_rng_init(ctypes.byref(st), 1, 5, 4) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_rng_draw(None, None, 1) == _lib.ERR_INVALID_ARG


class _FakeLoss:
    """A stand-in sampled loss: counts update() calls (batch.h:50 calls the wrapped loss's update first)."""
    f64 = False
    fitted = None

    def __init__(self, n):
        self.n, self.updates = n, 0

    def samples(self):
        return self.n

    def update(self):
        self.updates += 1


def test_batch_construction_order_matches_reference():
    from bbm_amd import fit
    g = GOLDEN["indices"][0]
    inner = _FakeLoss(g["samples"])
    b = fit.Batch(g["batchsize"], inner, g["seed"])
    want = np.asarray(g["index"], np.uint64).reshape(g["updates"] + 1, g["batchsize"])
    assert inner.updates == 1 and b.samples() == g["batchsize"]
    np.testing.assert_array_equal(b.index, want[0])
    for u in range(1, g["updates"] + 1):
        b.update()
        assert inner.updates == u + 1
        np.testing.assert_array_equal(b.index, want[u])
    assert b(g["batchsize"]) == 0.0 and b(-1) == 0.0     # idx outside the batch: masked (batch.h:66-67)


def test_gather_and_comm_validation(lib):
    from bbm_amd import _lib
    idx = np.zeros(4, np.uint64)
    p = (ctypes.c_void_p * 16)()
    assert lib.bbm_hip_gather_samples(idx.ctypes.data, 4, 10, p, p, 0, None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_gather_samples(idx.ctypes.data, 4, 10, p, p, 17, None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_gather_samples(idx.ctypes.data, 4, 10, p, p, 3, None) == _lib.ERR_INVALID_ARG   # NULL arrays
    assert lib.bbm_hip_gather_samples_f64(None, 4, 10, p, p, 3, None) == _lib.ERR_INVALID_ARG
    uid = (ctypes.c_uint8 * 128)()
    h = ctypes.c_void_p()
    assert lib.bbm_hip_comm_unique_id(uid, 64) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_comm_init(uid, 128, 2, 2, ctypes.byref(h)) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_comm_init(uid, 128, 0, 0, ctypes.byref(h)) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_comm_init(uid, 100, 0, 1, ctypes.byref(h)) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_comm_init(uid, 128, 0, 1, None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_comm_destroy(None) == _lib.OK
    assert lib.bbm_hip_comm_rank(None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_allreduce_sums(None, None, 1, None) == _lib.ERR_INVALID_ARG
    from bbm_amd import comm
    with pytest.raises(ValueError):
        comm.Comm(b"short", 0, 1)
