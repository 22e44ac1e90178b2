"""bbm::batch and the C-ABI's RCCL reduction on the GPU (run with -m gpu on an MI355X):

* batch::operator()(idx) (include/bbm/batch.h:64-70) -- the loss of each drawn sample -- equals the reference's own
  bbm::batch over its sampledlossfunction (tests/golden/batch.json, and the reference live) at 1e-5 per sample, after
  construction and after every update(); the masked index samples() gives 0 as in the reference;
* the batch's per-probe sums (all probes in one launch over the gathered samples) equal the reference's per-sample
  losses at the drawn indices summed in double, and equal one-probe launches bit for bit;
* a compass search over a batch redraws the batch every step (compass.h:103) and scores every probe of a step on
  that step's batch;
* a one-rank RCCL communicator of the C-ABI (bbm_hip_comm_init / bbm_hip_allreduce_sums) leaves the sums unchanged,
  and a sharded batch reduced through it equals the unsharded one.
Tolerance (north_star): 1e-5 relative.
"""
import numpy as np
import pytest

from tests import oracle_util as ou

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

META_FIT, FIT = ou.golden_fit()
GOLDEN = ou.golden_batch()
REL = 1e-5


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd


def _lin(grid):
    from bbm_amd import fit
    return fit.spherical_linearizer(grid["samples_in"], grid["samples_out"], grid["start_in"], grid["end_in"],
                                    grid["start_out"], grid["end_out"])


def _loss(bbm, name, grid="grid0", kind=3):
    from bbm_amd import fit
    fitted = bbm.BsdfModel(name)
    fitted.set_parameter_values(FIT[f"{name}_fitted"])
    reference = bbm.BsdfModel(name)
    reference.set_parameter_values(FIT[f"{name}_reference"])
    return fit.SampledLoss(fitted, reference, kind, _lin(META_FIT["grids"][grid]))


def _close(got, want):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    zero = want == 0
    assert np.all(got[zero] == 0), "masked / zero-loss samples must be exactly 0"
    rel = np.abs(got[~zero] - want[~zero]) / np.abs(want[~zero])
    assert rel.size == 0 or rel.max() <= REL, f"max rel {rel.max():.3e}"


@pytest.mark.parametrize("case", range(len(GOLDEN["losses"])))
def test_batch_per_sample_losses_match_reference(bbm, case):
    from bbm_amd import fit
    g = GOLDEN["losses"][case]
    lf = _loss(bbm, g["model"], g["grid"], g["loss"])
    b = fit.Batch(g["batchsize"], lf, g["seed"])
    want = np.asarray(g["per_sample"], np.float32).reshape(g["updates"] + 1, g["batchsize"])
    for u in range(g["updates"] + 1):
        if u:
            b.update()
        got = [b(i) for i in range(g["batchsize"])]
        _close(got, want[u])
    assert b(g["batchsize"]) == 0.0


def test_batch_probe_sums_match_reference(bbm):
    from bbm_amd import fit
    name = "Aggregate<Lambertian,Bagher>"
    grid = META_FIT["grids"]["grid0"]
    lf = _loss(bbm, name)
    b = fit.Batch(300, lf, seed=123)
    rng = np.random.default_rng(3)
    base = lf.fitted.parameter_values()
    probes = np.stack([base] + [base * rng.uniform(0.9, 1.1, base.size).astype(np.float32) for _ in range(11)])
    d = FIT["grid0_dirs"]
    for _ in range(3):
        got = b.probe_sums(probes).cpu().numpy()
        single = np.array([b.probe_sums(p[None]).cpu().numpy()[0] for p in probes])
        np.testing.assert_array_equal(got, single)          # one launch for all probes == one launch per probe
        idx = b.index[b.index < grid["size"]].astype(np.int64)
        for p, s in zip(probes, got):
            per = ou.ref_pair_losses(name, p, FIT[f"{name}_reference"], d[:3][:, idx], d[3:][:, idx], 3)
            want = np.sum(per.astype(np.float64))
            assert abs(s - want) <= REL * abs(want), f"{s} vs {want}"
        losses = b.probe_losses(probes)
        np.testing.assert_allclose(losses, (got / 300).astype(np.float32), rtol=0)
        b.update()


def test_compass_redraws_the_batch_each_step(bbm):
    from bbm_amd import fit
    name = "Aggregate<Lambertian,CookTorrance>"
    lf = _loss(bbm, name)
    b = fit.Batch(256, lf, seed=9)
    seen = [b.index.copy()]
    opt = fit.Compass(b, lf.fitted)
    seen.append(b.index.copy())                              # reset(): update() then the loss (compass.h:145-152)
    rng = fit.BatchRng(9, 0, lf.samples())
    for k in range(len(seen)):
        np.testing.assert_array_equal(seen[k], rng.draw(256))
    moved = 0
    for _ in range(6):
        step = opt.step_size
        e = opt.step()
        np.testing.assert_array_equal(b.index, rng.draw(256))   # the step's own batch
        # an accepted probe (the step size kept: expansion 1) is the batch mean at the new parameters, on that batch
        # (a rejected step keeps the previous batch's loss and only the probe / restore round-off of the parameters)
        if opt.step_size == step:
            moved += 1
            assert abs(e - b.loss_value()) <= 1e-6 * abs(e)
    assert moved > 0


def test_comm_one_rank_allreduce_is_identity(bbm):
    from bbm_amd import comm, fit
    uid = comm.unique_id()
    assert len(uid) == 128
    c = comm.Comm(uid, 0, 1)
    assert c.rank == 0 and c.size == 1
    lf = _loss(bbm, "Aggregate<Lambertian,Bagher>")
    probes = np.stack([lf.fitted.parameter_values(), FIT["Aggregate<Lambertian,Bagher>_reference"]])
    sums = lf.local_sums(probes)
    want = sums.cpu().numpy().copy()
    c.allreduce_sums(sums)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(sums.cpu().numpy(), want)
    # shards of a batch reduced through the communicator == the whole batch
    b = fit.Batch(500, lf, seed=77)
    whole = b.probe_sums(probes).cpu().numpy()
    parts = torch.zeros(2, dtype=torch.float64, device="cuda")
    for r in range(3):
        lo, hi = fit.shard_range(lf.samples(), r, 3)
        part = fit.SampledLoss(lf.fitted, lf.ref, 3, lf.lin)
        part.begin, part.n = lo, hi - lo
        part.pairs = lf.lin.directions(lo, hi - lo)
        part.ref = lf.ref[:, lo:hi].contiguous()
        pb = fit.Batch.__new__(fit.Batch)
        pb.loss, pb.f64, pb.index, pb._gathered, pb.batchsize = part, False, b.index, None, b.batchsize
        parts += pb.probe_sums(probes)
    c.allreduce_sums(parts)
    got = parts.cpu().numpy()
    assert np.all(np.abs(got - whole) <= 1e-12 * np.abs(whole))
    c.close()
