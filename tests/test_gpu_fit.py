"""Fitting path on the GPU (run with -m gpu on an MI355X), through the C-ABI (bbm_hip_linearize,
bbm_hip_loss) against the reference's own results:

* spherical linearizer directions == the reference's (tests/golden/fit.npz);
* MERL grid: every GPU direction pair maps back to its own index through the reference's
  merl_linearizer inverse map (the reference's forward map does not compile, see oracle/ref_fit.cpp);
* multi-probe loss sums == the reference's per-sample losses summed in double (1e-5 relative), for all
  six sample losses, and == its serial float total within float summation error;
* the batched compass follows the reference compass trajectory;
* determinism and shard additivity of the loss reduction.
Tolerance (north_star): 1e-5 relative for floating-point results.
"""
import numpy as np
import pytest

from tests import oracle_util as ou

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

META_FIT, FIT = ou.golden_fit()
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


def _model(bbm, name, params):
    m = bbm.BsdfModel(name)
    m.set_parameter_values(params)
    return m


@pytest.mark.parametrize("gname", sorted(META_FIT["grids"]))
def test_spherical_linearizer_matches_reference(bbm, gname):
    grid = META_FIT["grids"][gname]
    lin = _lin(grid)
    assert lin.size() == grid["size"]
    din, dout = lin.directions()
    got = torch.cat([din, dout]).cpu().numpy()
    ref = FIT[f"{gname}_dirs"]
    ulp = ou.ulp_diff(got, ref)
    assert ulp.max() <= 1, f"max ulp {ulp.max()}"
    assert np.mean(ulp == 0) > 0.999


def test_merl_linearizer_round_trips_through_reference_inverse(bbm):
    """The MERL grid (90 x 90 x 180): (1) GPU directions == the forward map evaluated in float64 within
    float round-off; (2) the reference's inverse map sends them back to their own index.  Every MERL
    sample sits exactly on the lower edge of its bin (idx / samples, merl_linearizer.h:74-75), so the
    inverse's floor(x + Epsilon) (:116-117) flips to the bin below whenever float round-off of the
    round trip exceeds Epsilon: the reference loses the same samples on the float64 directions rounded
    to float, and a flip is never more than one bin."""
    from bbm_amd import fit
    lin = fit.merl_linearizer()
    n = lin.size()
    assert n == 90 * 90 * 180
    din, dout = lin.directions()
    din, dout = din.cpu().numpy(), dout.cpu().numpy()
    rin, rout = ou.merl_directions_f64()
    err = max(np.abs(din - rin).max(), np.abs(dout - rout).max())
    assert err <= 2e-6, f"forward map off by {err}"
    idx = ou.ref_merl_index(din, dout).astype(np.int64)
    idx64 = ou.ref_merl_index(rin.astype(np.float32), rout.astype(np.float32)).astype(np.int64)
    want = np.arange(n, dtype=np.int64)
    td, th = (want // 180) % 90, want // (180 * 90)
    # well-posed samples: phi_d defined (theta_d > 0) and both directions strictly above the horizon
    ok = (td > 0) & (din[2] > 1e-3) & (dout[2] > 1e-3)
    frac, frac64 = np.mean(idx[ok] == want[ok]), np.mean(idx64[ok] == want[ok])
    assert frac > 0.975 and frac >= frac64 - 0.005, f"round trip {frac:.5f} (float64 directions: {frac64:.5f})"
    bad = ok & (idx != want)
    dth = idx[bad] // (180 * 90) - th[bad]
    dtd = (idx[bad] // 180) % 90 - td[bad]
    dpd = (idx[bad] % 180 - want[bad] % 180 + 90) % 180 - 90          # phi_d is cyclic
    assert np.all(np.abs(dth) <= 1) and np.all(np.abs(dtd) <= 1) and np.all(np.abs(dpd) <= 1)
    # theta_d == 0 (in == out): the inverse map sets phi_d = 0 (merl_linearizer.h:110-111)
    sel = (td == 0) & (din[2] > 1e-3)
    assert np.all(idx[sel] == (th[sel] * 90 * 180))


def _loss_case(bbm, name, gname, kind):
    from bbm_amd import fit
    grid = META_FIT["grids"][gname]
    fitted = _model(bbm, name, FIT[f"{name}_fitted"])
    reference = _model(bbm, name, FIT[f"{name}_reference"])
    return fit.SampledLoss(fitted, reference, kind, _lin(grid))


@pytest.mark.parametrize("name", ["Aggregate<Lambertian,Bagher>", "Aggregate<Lambertian,CookTorrance>"])
@pytest.mark.parametrize("gname", ["grid0", "grid1"])
@pytest.mark.parametrize("kind", range(6))
def test_loss_matches_reference(bbm, name, gname, kind):
    loss = _loss_case(bbm, name, gname, kind)
    per = FIT[f"{name}_{gname}_loss{kind}"]
    want = np.sum(per.astype(np.float64))
    s = float(loss.probe_sums(loss.fitted._params[None]).cpu().numpy()[0])
    assert abs(s - want) <= REL * abs(want), f"{s} vs {want}"
    # the reference's own serial float total (sampledlossfunction.h:80-87): float summation error
    total = META_FIT["loss"][f"{name}_{gname}_loss{kind}"]
    assert abs(s / per.size - total) <= 1e-4 * abs(total)


def test_multi_probe_batch_equals_single_probes(bbm):
    name = "Aggregate<Lambertian,Bagher>"
    loss = _loss_case(bbm, name, "grid0", 3)
    rng = np.random.default_rng(7)
    base = loss.fitted.parameter_values()
    probes = np.stack([base] + [base * rng.uniform(0.8, 1.2, base.size).astype(np.float32) for _ in range(20)] +
                      [FIT[f"{name}_reference"]])
    batch = loss.probe_sums(probes).cpu().numpy()
    single = np.array([loss.probe_sums(p[None]).cpu().numpy()[0] for p in probes])
    np.testing.assert_array_equal(batch, single)          # batching changes nothing, not even rounding
    assert batch[-1] == 0.0                               # fitted == reference: every sample loss is 0
    again = loss.probe_sums(probes).cpu().numpy()
    np.testing.assert_array_equal(batch, again)           # deterministic


def test_probe_losses_against_reference_per_probe(bbm):
    """Random probes: GPU sums vs the reference's per-sample losses for the same parameters."""
    name = "Aggregate<Lambertian,CookTorrance>"
    loss = _loss_case(bbm, name, "grid0", 3)
    d = FIT["grid0_dirs"]
    rng = np.random.default_rng(11)
    base = loss.fitted.parameter_values()
    lo, hi = loss.fitted.parameter_lower_bound(), loss.fitted.parameter_upper_bound()
    probes = np.stack([np.clip(base * rng.uniform(0.5, 1.5, base.size).astype(np.float32), lo, hi) for _ in range(12)])
    got = loss.probe_sums(probes).cpu().numpy()
    for p, g in zip(probes, got):
        want = np.sum(ou.ref_pair_losses(name, p, FIT[f"{name}_reference"], d[:3], d[3:], 3).astype(np.float64))
        assert abs(g - want) <= REL * abs(want)


def test_merl_grid_loss_matches_reference_per_sample(bbm):
    """Full MERL grid (1.458 M pairs, BASELINE config 5): GPU loss vs the reference's per-sample losses on
    the same direction pairs, double sums, 1e-5."""
    from bbm_amd import fit
    name = "Aggregate<Lambertian,Bagher>"
    fitted = _model(bbm, name, FIT[f"{name}_fitted"])
    reference = _model(bbm, name, FIT[f"{name}_reference"])
    lin = fit.merl_linearizer()
    loss = fit.SampledLoss(fitted, reference, "standardLog", lin)
    got = float(loss.probe_sums(fitted._params[None]).cpu().numpy()[0])
    din, dout = lin.directions()
    per = ou.ref_pair_losses(name, fitted._params, reference._params, din.cpu().numpy(), dout.cpu().numpy(), 3)
    want = np.sum(per.astype(np.float64))
    assert abs(got - want) <= REL * abs(want), f"{got} vs {want}"


def test_shard_sums_add_up(bbm):
    from bbm_amd import fit
    name = "Aggregate<Lambertian,Bagher>"
    fitted = _model(bbm, name, FIT[f"{name}_fitted"])
    reference = _model(bbm, name, FIT[f"{name}_reference"])
    lin = fit.merl_linearizer()
    whole = fit.SampledLoss(fitted, reference, 0, lin).probe_sums(fitted._params[None]).cpu().numpy()[0]

    parts = []
    for r in range(4):
        l = fit.SampledLoss(fitted, reference, 0, lin)
        b, e = fit.shard_range(lin.size(), r, 4)
        l.begin, l.n = b, e - b
        l.pairs = lin.directions(b, e - b)
        l.ref = fit.reference_table(reference, lin, b, e - b)
        parts.append(l.probe_sums(fitted._params[None]).cpu().numpy()[0])
    assert abs(sum(parts) - whole) <= 1e-12 * abs(whole)


@pytest.mark.parametrize("ci", range(len(META_FIT["compass"])))
def test_compass_on_gpu_follows_reference(bbm, ci):
    from bbm_amd import fit
    run = META_FIT["compass"][ci]
    name, grid = run["model"], META_FIT["grids"][run["grid"]]
    fitted = bbm.BsdfModel(name)
    reference = _model(bbm, name, FIT[f"{name}_reference"])
    loss = fit.SampledLoss(fitted, reference, run["loss"], _lin(grid))
    opt = fit.Compass(loss, fitted)
    assert abs(opt.loss_value - run["loss0"]) <= 1e-5 * run["loss0"]
    ref_params, ref_loss = FIT[f"compass{ci}_params"], FIT[f"compass{ci}_loss"]
    same = 0
    for t in range(run["steps"]):
        e = opt.step()
        if np.array_equal(fitted.parameter_values(fit.ALL), ref_params[t]):
            same += 1
        else:
            break
        assert abs(e - ref_loss[t]) <= 1e-5 * ref_loss[t] + 1e-9
    # identical decisions unless two probes tie within float summation error (then both paths are valid)
    assert same == run["steps"], f"diverged at step {same}"


@pytest.mark.parametrize("lin_kind", ["merl", "grid1"])
def test_materialized_pairs_equal_computed_linearizer(bbm, lin_kind):
    """bbm_hip_loss_pairs over the materialised pairs == bbm_hip_loss computing the linearizer in-kernel,
    bit for bit (the pairs come from the same device code)."""
    from bbm_amd import fit
    name = "Aggregate<Lambertian,Bagher>"
    fitted = _model(bbm, name, FIT[f"{name}_fitted"])
    reference = _model(bbm, name, FIT[f"{name}_reference"])
    lin = fit.merl_linearizer() if lin_kind == "merl" else _lin(META_FIT["grids"][lin_kind])
    a = fit.SampledLoss(fitted, reference, "standardLog", lin, materialize=True)
    b = fit.SampledLoss(fitted, reference, "standardLog", lin, materialize=False)
    probes = np.stack([fitted._params, reference._params, fitted._params * np.float32(1.01)])
    np.testing.assert_array_equal(a.probe_sums(probes).cpu().numpy(), b.probe_sums(probes).cpu().numpy())
