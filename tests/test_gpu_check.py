"""checkBsdf statistics on the GPU (bbm_hip_check through bbm_amd.check; run with -m gpu) against
the reference recomputing the same statistic from the same random draws (tests/check_oracle.py).

Tolerances (north_star: 1e-5 relative for floating point):
  * sums of per-sample terms: 1e-5 relative to the sum of their magnitudes -- per-sample terms agree
    to a few ulp (eval / pdf parity), sampled directions to ~1e-6 (see test_gpu_parity's sample tests);
  * counts (accepted samples, negative pdfs, below-horizon samples): exact, except histogram bins, where
    a sample within ~1e-6 of a bin edge may land in the neighbour bin (L1 difference <= 1e-3 of the total);
  * draws: bit-exact with the numpy restatement.
"""
import numpy as np
import pytest

from tests import check_oracle as co
from tests import oracle_util as ou

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(ou.ref() is None, reason="reference shim not built")]

SEED = 20241
MODELS = ["Lambertian", "CookTorrance", "GGX", "Ward", "AshikhminShirleyFull", "LowSmooth", "OrenNayar",
          "Aggregate<Lambertian,Bagher>", "RibardiereAnisotropic", "NganLafortune", "EPD", "He", "NganHe"]


@pytest.fixture(scope="module")
def chk():
    import bbm_amd
    from bbm_amd import check
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd, check


def _model(bbm, name):
    m = bbm.BsdfModel(name)
    if name == "CookTorrance":
        m.set_parameter_values(np.array([0.6, 0.4, 0.3, 0.3, 1.6], np.float32))
    return m


def _close(got, want, scale, rel=1e-5, what=""):
    if np.isnan(want):   # the reference's own statistic is NaN (e.g. He's G at in == out, theta 0)
        assert np.isnan(got), f"{what}: {got} vs NaN"
        return
    assert abs(got - want) <= rel * scale + 1e-30, f"{what}: {got} vs {want} (scale {scale})"


@pytest.mark.parametrize("test,slot,draw,offset", [(0, 0, 0, 0), (1, 0, 1, 12345), (5, 77, 0, 3), (3, 0, 2, 1 << 33)])
def test_draws_bit_exact(chk, test, slot, draw, offset):
    _, check = chk
    got = check.draws(test, SEED, slot, draw, offset, 4099).cpu().numpy()
    np.testing.assert_array_equal(got, co.draws(test, SEED, slot, draw, offset, 4099))


def test_sphere_and_trial_directions(chk):
    bbm, check = chk
    lib = bbm._lib.load()
    xi = co.draws(0, SEED, 0, 0, 0, 100_000)
    for hemi in (0, 1):
        want, _ = co.sphere_dirs(xi, hemisphere=bool(hemi))
        u = torch.from_numpy(xi).cuda()
        d = torch.empty((3, xi.shape[1]), dtype=torch.float32, device="cuda")
        bbm._lib.check(lib.bbm_hip_sphere_dirs(u[0].data_ptr(), u[1].data_ptr(), xi.shape[1], hemi, d[0].data_ptr(),
                                               d[1].data_ptr(), d[2].data_ptr(), None))
        torch.cuda.synchronize()
        assert np.abs(d.cpu().numpy() - want).max() <= 2.5e-7
    for sphere in (False, True):
        got = check.trial_directions(check.PDFINT, SEED, 16, sphere).cpu().numpy()
        assert np.abs(got - co.trial_dirs(check.PDFINT, SEED, 16, sphere)).max() <= 2.5e-7


@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("importance", [False, True])
def test_reflectance_matches_reference(chk, name, importance):
    bbm, check = chk
    m = _model(bbm, name)
    n = 200_000
    outs = check.reflectance_outs(3)
    acc = check.run(m, check.REFLECTANCE, n, 3, torch.from_numpy(outs).cuda(), SEED, importance=importance)
    for t in range(3):
        want = co.reflectance(name, m.parameter_values(), outs[:, t], n, SEED, t, importance)
        assert abs(acc[t, 3] - want[3]) <= 2, f"{name} accepted {acc[t, 3]} vs {want[3]}"
        scale = max(abs(want[:3]).max(), 1e-12)
        for c in range(3):
            _close(acc[t, c], want[c], scale, 2e-5 if importance else 1e-5, f"{name} theta {t} ch {c}")


@pytest.mark.parametrize("test", ["reflectance", "pdf", "count"])
def test_exact_sampling_twin_matches_reference(chk, test):
    """Exact mode launches the sampling tests on the sampler's twin (glibc erff / logf in Beckmann's visible-normal
    sampler, math.hpp exact_sample_t): importance-sampled reflectance, the pdf test and the sample histogram still
    equal the reference's to the same bars as the default sampler."""
    bbm, check = chk
    m = _model(bbm, "CookTorrance")
    p = m.parameter_values()
    bbm.set_exact_subnormals(True)
    try:
        if test == "reflectance":
            n = 200_000
            outs = check.reflectance_outs(3)
            acc = check.run(m, check.REFLECTANCE, n, 3, torch.from_numpy(outs).cuda(), SEED, importance=True)
            for t in range(3):
                want = co.reflectance("CookTorrance", p, outs[:, t], n, SEED, t, True)
                assert abs(acc[t, 3] - want[3]) <= 2
                scale = max(abs(want[:3]).max(), 1e-12)
                for c in range(3):
                    _close(acc[t, c], want[c], scale, 2e-5, f"exact theta {t} ch {c}")
        elif test == "pdf":
            n = 100_000
            acc = check.run(m, check.PDF, n, 1, None, SEED, sphere=False)[0]
            for j, (neg, below, mism) in enumerate(co.pdf_test("CookTorrance", p, n, SEED, False)):
                assert acc[j] == neg and abs(acc[2 + j] - below) <= 2
                assert abs(acc[4 + j] - mism) <= 1e-3 * mism + 1e-5 * n
        else:
            th, ph, trials, ns = 6, 10, 2, 50_000
            t = check.trial_directions(check.SAMPLE_COUNT, SEED, trials)
            counts = check.run(m, check.SAMPLE_COUNT, ns, trials, t, SEED, bins=(th, ph))
            tn = t.cpu().numpy()
            for k in range(trials):
                wc = co.sample_count("CookTorrance", p, tn[:, k], k, ns, SEED, th, ph)
                assert counts[k].sum() == wc.sum()
                assert np.abs(counts[k] - wc).sum() <= max(2, 1e-3 * wc.sum()), (counts[k], wc)
    finally:
        bbm.set_exact_subnormals(False)


@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("test", [1, 2])
def test_reciprocity_and_adjoint_match_reference(chk, name, test):
    bbm, check = chk
    m = _model(bbm, name)
    n = 100_000
    acc = check.run(m, test, n, 1, None, SEED)[0]
    sums, hmax, k = co.symmetry(name, m.parameter_values(), n, SEED, test)
    # scale: the magnitude of the evaluated values (differences of a reciprocal model are round-off)
    din, _ = co.sphere_dirs(co.draws(test, SEED, 0, 0, 0, n))
    dout, _ = co.sphere_dirs(co.draws(test, SEED, 0, 1, 0, n))
    f = np.abs(ou.ref_eval_pdf(name, m.parameter_values(), din, dout, nthreads=8)[:3]).astype(np.float64)
    scale = f.sum()
    for c in range(3):
        _close(acc[c], sums[c], scale, 1e-5, f"{name} sum {c}")
        if test == 1:
            assert acc[3 + c] == acc[c]
    # the largest difference: each value is within 1e-5 of the reference's, so the maximum is within
    # 1e-5 of the largest value's magnitude (a non-reciprocal model's maximum need not be unique)
    assert abs(max(acc[8], 0.0) - hmax) <= 2e-5 * f.sum(axis=0).max() + 1e-6 * hmax, (acc[8], hmax)


@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("sphere", [False, True])
def test_pdf_properties_match_reference(chk, name, sphere):
    bbm, check = chk
    m = _model(bbm, name)
    n = 100_000
    acc = check.run(m, check.PDF, n, 1, None, SEED, sphere=sphere)[0]
    want = co.pdf_test(name, m.parameter_values(), n, SEED, sphere)
    for j, (neg, below, mism) in enumerate(want):
        assert acc[j] == neg and abs(acc[2 + j] - below) <= 2, (name, j, acc[:6], want)
        # |sample.pdf - pdf|: round-off for most models (then only bounded); AshikhminShirleyFull's
        # one-sample mixture reports a pdf mixing two candidates (ashikhminshirleyfull.h:96-124), a real
        # difference the GPU must reproduce
        assert abs(acc[4 + j] - mism) <= 1e-3 * mism + 1e-5 * n, (name, acc[4 + j], mism)


@pytest.mark.parametrize("name", MODELS)
def test_pdf_integral_matches_reference(chk, name):
    bbm, check = chk
    m = _model(bbm, name)
    n = 200_000
    t = check.trial_directions(check.PDFINT, SEED, 4)
    acc = check.run(m, check.PDFINT, n, 4, t, SEED)
    tn = t.cpu().numpy()
    for k in range(4):
        want = co.pdf_int(name, m.parameter_values(), tn[:, k], n, SEED, k)
        _close(acc[k, 0], want, abs(want), 1e-5, f"{name} trial {k}")
        assert acc[k, 1] == acc[k, 0]


@pytest.mark.parametrize("name", ["Lambertian", "CookTorrance", "Ward", "Aggregate<Lambertian,Bagher>", "LowSmooth", "EPD",
                                  "HeWestin"])
def test_chi2_pdf_bins_and_histogram_match_reference(chk, name):
    bbm, check = chk
    m = _model(bbm, name)
    th, ph, trials, ps, ns = 6, 10, 2, 256, 50_000
    bins = th * ph
    t = check.trial_directions(check.SAMPLE_COUNT, SEED, trials)
    pdf = check.run(m, check.SAMPLE_PDF, ps, trials * bins, t, SEED, bins=(th, ph))[:, 0].reshape(trials, bins)
    counts = check.run(m, check.SAMPLE_COUNT, ns, trials, t, SEED, bins=(th, ph))
    tn = t.cpu().numpy()
    for k in range(trials):
        want = co.sample_pdf(name, m.parameter_values(), tn[:, k], k, bins, ps, SEED, th, ph)
        scale = np.abs(want).sum()
        assert np.abs(pdf[k] - want).max() <= 1e-5 * scale + 1e-30, name
        wc = co.sample_count(name, m.parameter_values(), tn[:, k], k, ns, SEED, th, ph)
        assert counts[k].sum() == wc.sum()
        assert np.abs(counts[k] - wc).sum() <= max(2, 1e-3 * wc.sum()), (name, counts[k], wc)


def test_shards_merge_to_the_single_gpu_result(chk):
    bbm, check = chk
    m = _model(bbm, "CookTorrance")
    n = 300_001
    whole = check.run(m, check.RECIPROCITY, n, 1, None, SEED)
    parts = []
    for r in range(3):
        b, e = check.shard_range(n, r, 3)
        parts.append(check.run(m, check.RECIPROCITY, e - b, 1, None, SEED, begin=b))
    merged = check.merge_acc(parts)
    np.testing.assert_allclose(merged[:, :8], whole[:, :8], rtol=1e-12)
    assert tuple(merged[0, 8:12]) == tuple(whole[0, 8:12])
    t = check.trial_directions(check.SAMPLE_COUNT, SEED, 2)
    c = check.run(m, check.SAMPLE_COUNT, n, 2, t, SEED, bins=(5, 7))
    c2 = sum(check.run(m, check.SAMPLE_COUNT, e - b, 2, t, SEED, bins=(5, 7), begin=b)
             for b, e in (check.shard_range(n, r, 2) for r in range(2)))
    np.testing.assert_array_equal(c, c2)


def test_deterministic(chk):
    bbm, check = chk
    m = _model(bbm, "GGX")
    outs = torch.from_numpy(check.reflectance_outs(2)).cuda()
    a = check.run(m, check.REFLECTANCE, 1_000_003, 2, outs, SEED, importance=True)
    b = check.run(m, check.REFLECTANCE, 1_000_003, 2, outs, SEED, importance=True)
    np.testing.assert_array_equal(a, b)


def test_cli_runs_every_test(chk, capsys):
    _, check = chk
    model = "CookTorrance(albedo=[0.5,0.5,0.5], roughness=0.3, eta=1.5)"
    assert check.main([f"bsdfmodel={model}", "test=reflectance", "samples=100000", "theta=3", "importanceSampling"]) == 0
    assert check.main([f"bsdfmodel={model}", "test=reciprocity", "samples=100000"]) == 0
    assert check.main([f"bsdfmodel={model}", "test=adjoint", "samples=100000"]) == 0
    assert check.main([f"bsdfmodel={model}", "test=pdf", "samples=100000", "checkBelowHorizon"]) == 0
    assert check.main([f"bsdfmodel={model}", "test=pdfInt", "samples=100000", "trials=3"]) == 0
    assert check.main([f"bsdfmodel={model}", "test=sample", "pdfSamples=256", "samples=100000", "trials=2"]) == 0
    out = capsys.readouterr().out
    for line in ("Reflectance test with 3 directions", "Radiance   average", "Importance average",
                 "Adjoint difference average", "PDF has 0/0 negative PDF values", "Integral = ", "Chi2 for ", "P = "):
        assert line in out, line
    print(out)


def test_importance_sampled_reflectance_estimates_reflectance(chk):
    """The MC estimate converges to the model's reflectance where the reference's reflectance is exact
    (Lambertian albedo; AshikhminShirleyFull's diffuse + specular approximation within a few %)."""
    bbm, check = chk
    res = check.test_reflectance(bbm.Lambertian(), samples=1_000_000, theta=4, importanceSampling=True, verbose=False)
    np.testing.assert_allclose(res["estimate"], res["reflectance"], rtol=2e-3)
