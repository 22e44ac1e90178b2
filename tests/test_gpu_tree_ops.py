"""The fitting loss and checkBsdf for ANY model and for doubleRGB (bbm_hip_loss_tree(_f64), bbm_hip_check_tree(_f64);
bbm_amd.fit.SampledLoss / bbm_amd.check.run on AggregateModels and with f64=True).  The reference takes any
bsdfmodel and any configuration there: sampledlossfunction<BSDF, ...> (include/bbm/sampledlossfunction.h:34,
:62-87), compass (include/optimizer/compass.h:40-80) and checkBsdf of any bsdf_import string
(bin/checkBsdf.cpp:435-479).  Checked against the reference recomputing the same quantities (oracle/_ref): its
aggregatemodel types and per-sample losses, its runtime aggregatebsdf (oracle/ref_runtime.cpp) and its doubleRGB
models; statistics from the same draws (tests/check_oracle.py)."""
import numpy as np
import pytest

from tests import check_oracle as co
from tests import oracle_util as ou
from tests import test_gpu_runtime as tr

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(ou.ref() is None, reason="reference shim not built")]

SEED = 20241
REL = 1e-5
THREE = "Aggregate(Lambertian(albedo = [0.2, 0.3, 0.4]), CookTorrance(roughness = 0.3), GGX(roughness = 0.15))"


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd


def _pairs(bbm, n, seed=0xF17):
    return (bbm.fill_directions(seed, 0, 0, n, mode=0), bbm.fill_directions(seed, 1, 0, n, mode=0))


def _np_loss(kind, din, dout, v, r):
    """The six per-sample losses (include/loss/cosine_weighted_{l2,log}.h) in numpy, in v's dtype: float32 per
    operation as the reference's floatRGB (log: numpy's, within an ulp of logf), or float64 (doubleRGB)."""
    dt = v.dtype
    c = np.maximum(din[2], dt.type(0))
    si = np.sqrt(np.maximum(dt.type(1) - din[2] * din[2], dt.type(0)))
    so = np.sqrt(np.maximum(dt.type(1) - dout[2] * dout[2], dt.type(0)))
    co_ = np.maximum(dout[2], dt.type(0))
    if kind <= 2:
        e = ((v - r) * c).astype(np.float64)
    else:
        e = (np.log(dt.type(1) + v * c) - np.log(dt.type(1) + r * c)).astype(np.float64)
    h = (e * e).sum(0)
    if kind in (1, 4):
        out = h * si
    elif kind in (2, 5):
        out = ((h * co_) * si) * so
    else:
        out = (h * si) * so
    return out.astype(dt)


def _composed_ct(bbm):
    lam, ct = bbm.Lambertian(albedo=[0.2, 0.3, 0.4]), bbm.CookTorrance(albedo=[0.6, 0.5, 0.4], roughness=0.25, eta=1.6)
    return lam, ct


@pytest.mark.parametrize("kind", [0, 3, 5])
def test_tree_loss_equals_fused_loss(bbm, kind):
    """Aggregate(Lambertian, CookTorrance) composed (bbm_hip_loss_tree) and fused (bbm_hip_loss_pairs): two children
    evaluate to the same floats, so the per-probe sums agree to the summation order (~1e-15)."""
    from bbm_amd import fit
    lam, ct = _composed_ct(bbm)
    fused = bbm.Aggregate(lam, ct)
    composed = bbm.Aggregate(lam, ct, fused=False)
    assert isinstance(composed, bbm.AggregateModel)
    lin = fit.spherical_linearizer((45, 30), (45, 30))
    ref = bbm.fromString(tr.STRINGS["fused_ct"].replace("0.25", "0.3"))
    a = fit.SampledLoss(fused, ref, kind, lin)
    b = fit.SampledLoss(composed, ref, kind, lin)
    assert b.tree and not a.tree
    rng = np.random.default_rng(3)
    base = fused.parameter_values()
    probes = np.stack([base] + [base * rng.uniform(0.8, 1.2, base.size).astype(np.float32) for _ in range(7)])
    sa, sb = a.probe_sums(probes).cpu().numpy(), b.probe_sums(probes).cpu().numpy()
    np.testing.assert_allclose(sb, sa, rtol=1e-12, atol=0)


@pytest.mark.parametrize("kind", [0, 3])
def test_tree_loss_three_children_vs_reference(bbm, kind):
    """A three-child aggregatemodel (composed) and the runtime aggregate of the same string: the GPU's per-probe sums
    against the per-sample losses of the reference's own evaluation (aggregatemodel type / aggregatebsdf)."""
    from bbm_amd import fit
    n = 1 << 18
    din, dout = _pairs(bbm, n)
    hin, hout = din.cpu().numpy(), dout.cpu().numpy()
    rt = bbm.fromString(THREE)
    kids = [bbm.BsdfModel(c.name) for c in rt._children]
    for k, c in zip(kids, rt._children):
        k.set_parameter_values(c.parameter_values())
    tm = bbm.Aggregate(*kids)
    refm = bbm.CookTorrance(roughness=0.2)
    rv = ou.ref_eval_pdf("CookTorrance", refm.parameter_values(), hin, hout, nthreads=8)[:3]
    for model, fn in ((tm, lambda p: ou.ref_eval_pdf("Aggregate<Lambertian,CookTorrance,GGX>", p, hin, hout, nthreads=8)),
                      (rt, lambda p: ou.ref_runtime_eval_pdf(("Aggregate", [("Lambertian", p[:3]), ("CookTorrance", p[3:8]),
                                                                            ("GGX", p[8:])]), hin, hout))):
        loss = fit.SampledLoss(model, torch.from_numpy(rv).cuda(), kind, pairs=(din, dout))
        base = model.parameter_values()
        probes = np.stack([base, (base * np.float32(0.9)).astype(np.float32)])
        got = loss.probe_sums(probes).cpu().numpy()
        for p, g in zip(probes, got):
            want = _np_loss(kind, hin, hout, fn(p)[:3], rv).astype(np.float64).sum()
            assert abs(g - want) <= REL * abs(want), (model.name, g, want)


@pytest.mark.parametrize("key", ["single", "three"])
def test_tree_loss_f64_vs_reference(bbm, key):
    """doubleRGB: CookTorrance alone (a one-leaf tree) and the three-child runtime aggregate, per-sample losses in
    double against the reference's doubleRGB evaluation; then a compass in double moves downhill."""
    from bbm_amd import fit
    n = 1 << 18
    din, dout = _pairs(bbm, n)
    hin, hout = din.cpu().numpy().astype(np.float64), dout.cpu().numpy().astype(np.float64)
    if key == "single":
        model = bbm.CookTorrance(albedo=[0.3, 0.4, 0.5], roughness=0.3, eta=1.4)
        fn = lambda p: ou.ref_eval_pdf_dd("CookTorrance", np.asarray(p, np.float32), hin, hout, nthreads=8)  # noqa: E731
    else:
        model = bbm.fromString(THREE)
        fn = lambda p: ou.ref_runtime_eval_pdf(tr.tree_of(model), hin, hout, f64=True)  # noqa: E731
    rv = ou.ref_eval_pdf_dd("GGX", bbm.GGX(roughness=0.2).parameter_values(), hin, hout, nthreads=8)[:3]
    loss = fit.SampledLoss(model, torch.from_numpy(rv).cuda(), 3, f64=True, pairs=(din, dout))
    base = model.parameter_values().astype(np.float64)
    got = loss.probe_sums(base[None]).cpu().numpy()[0]
    want = _np_loss(3, hin, hout, fn(base)[:3], rv).sum()
    assert abs(got - want) <= 1e-11 * abs(want), (got, want)
    comp = fit.Compass(loss)
    assert comp.V is np.float64 and comp.parameters.dtype == np.float64
    l0 = comp.loss_value
    for _ in range(6):
        comp.step()
    assert comp.loss_value <= l0


def _check_models(bbm):
    rt = bbm.fromString(THREE)
    kids = [bbm.BsdfModel(c.name) for c in rt._children]
    for k, c in zip(kids, rt._children):
        k.set_parameter_values(c.parameter_values())
    composed = bbm.Aggregate(bbm.CookTorrance(roughness=0.3), bbm.GGX(roughness=0.15))
    return [("Aggregate<CookTorrance,GGX>", composed, composed.parameter_values()), (tr.tree_of(rt), rt, None)]


@pytest.mark.parametrize("which", [0, 1])
@pytest.mark.parametrize("importance", [False, True])
def test_tree_check_reflectance_vs_reference(bbm, which, importance):
    from bbm_amd import check
    name, m, params = _check_models(bbm)[which]
    n = 100_000
    outs = check.reflectance_outs(3)
    acc = check.run(m, check.REFLECTANCE, n, 3, torch.from_numpy(outs).cuda(), SEED, importance=importance)
    for t in range(3):
        want = co.reflectance(name, params, outs[:, t], n, SEED, t, importance)
        assert abs(acc[t, 3] - want[3]) <= 2
        scale = max(abs(want[:3]).max(), 1e-12)
        for c in range(3):
            assert abs(acc[t, c] - want[c]) <= 2e-5 * scale, (t, c, acc[t, c], want[c])


@pytest.mark.parametrize("which", [0, 1])
def test_tree_check_symmetry_pdf_pdfint_sample(bbm, which):
    from bbm_amd import check
    name, m, params = _check_models(bbm)[which]
    n = 50_000
    for test in (check.RECIPROCITY, check.ADJOINT):
        acc = check.run(m, test, n, 1, None, SEED)[0]
        sums, hmax, k = co.symmetry(name, params, n, SEED, test)
        for c in range(3):
            assert abs(acc[c] - sums[c]) <= 1e-5 * max(abs(sums).max(), 1e-12)
        assert abs(acc[8] - hmax) <= 1e-5 * max(hmax, 1e-12)
    acc = check.run(m, check.PDF, n, 1, None, SEED)[0]
    want = co.pdf_test(name, params, n, SEED, False)
    for j, (neg, below, absdiff) in enumerate(want):
        assert acc[j] == neg and acc[2 + j] == below
        assert abs(acc[4 + j] - absdiff) <= 1e-4 * max(absdiff, 1e-9) + 1e-6
    t = check.trial_directions(check.PDFINT, SEED, 4)
    acc = check.run(m, check.PDFINT, n, 4, t, SEED)
    for s in range(4):
        want = co.pdf_int(name, params, t[:, s].cpu().numpy(), n, SEED, s)
        assert abs(acc[s, 0] - want) <= 1e-5 * max(abs(want), 1e-12)
    theta, phi, trials = 4, 6, 2
    t = check.trial_directions(check.SAMPLE_COUNT, SEED, trials)
    counts = check.run(m, check.SAMPLE_COUNT, n, trials, t, SEED, bins=(theta, phi))
    for s in range(trials):
        want = co.sample_count(name, params, t[:, s].cpu().numpy(), s, n, SEED, theta, phi)
        assert np.abs(counts[s] - want).sum() <= 1e-3 * n
    pdfs = check.run(m, check.SAMPLE_PDF, 512, trials * theta * phi, t, SEED, bins=(theta, phi))
    for s in range(trials):
        want = co.sample_pdf(name, params, t[:, s].cpu().numpy(), s, theta * phi, 512, SEED, theta, phi)
        np.testing.assert_allclose(pdfs[s * theta * phi:(s + 1) * theta * phi, 0], want, rtol=1e-5, atol=1e-9)


def _sphere_dirs_d(xi):
    """sampleSphere in doubleRGB (checkBsdf.cpp:28-35): theta = safe_acos(1 - 2 xi0), phi = xi1 Pi(2), double."""
    x0, x1 = xi[0].astype(np.float64), xi[1].astype(np.float64)
    th = np.arccos(np.clip(1.0 - 2.0 * x0, -1.0, 1.0))
    ph = x1 * (2.0 * np.pi)
    return np.stack([np.cos(ph) * np.sin(th), np.sin(ph) * np.sin(th), np.cos(th)]), np.full(x0.size, 1.0 / (4 * np.pi))


@pytest.mark.parametrize("name", ["CookTorrance", "runtime"])
def test_tree_check_f64_vs_reference(bbm, name):
    """doubleRGB checkBsdf: the reflectance (importance sampled) and pdf-integral statistics of a single model and of
    the three-child runtime aggregate, every per-sample term in double, against the reference's doubleRGB objects
    from the same draws."""
    from bbm_amd import check
    n = 100_000
    if name == "CookTorrance":
        m = bbm.CookTorrance(albedo=[0.6, 0.4, 0.3], roughness=0.3, eta=1.6)
        p = m.parameter_values()
        tree = ("CookTorrance", p)          # a one-leaf tree: the reference's doubleRGB bsdf_ptr on double inputs
    else:
        m = bbm.fromString(THREE)
        tree = tr.tree_of(m)
    ev = lambda a, b: ou.ref_runtime_eval_pdf(tree, a, b, f64=True)  # noqa: E731
    smp = lambda o, x: ou.ref_runtime_sample(tree, o, x, f64=True)  # noqa: E731
    th = (np.arange(3) * (0.5 * np.pi)) / 3
    outs = np.stack([np.sin(th), 0.0 * th, np.cos(th)])
    acc = check.run(m, check.REFLECTANCE, n, 3, torch.from_numpy(outs).cuda(), SEED, importance=True, f64=True)
    for t in range(3):
        xi = co.draws(check.REFLECTANCE, SEED, t, 0, 0, n).astype(np.float64)
        o = np.repeat(outs[:, t:t + 1], n, axis=1)
        s, _ = smp(o, xi)
        f = ev(s[:3], o)[:3]
        ok = s[3] > np.finfo(np.float64).eps
        want = ((f[:, ok] * s[2, ok]) / s[3, ok]).sum(1)
        assert acc[t, 3] == ok.sum()
        np.testing.assert_allclose(acc[t, :3], want, rtol=1e-9)
    tr_dirs, _ = _sphere_dirs_d(np.concatenate([co.draws(check.PDFINT, SEED, k, 3, 0, 1) for k in range(2)], 1))
    acc = check.run(m, check.PDFINT, n, 2, torch.from_numpy(tr_dirs).cuda(), SEED, f64=True)
    for k in range(2):
        d, sp = _sphere_dirs_d(co.draws(check.PDFINT, SEED, k, 0, 0, n))
        pd = ev(d, np.repeat(tr_dirs[:, k:k + 1], n, axis=1))[3]
        np.testing.assert_allclose(acc[k, 0], (pd / sp).sum(), rtol=1e-9)


def test_tree_entry_points_refuse_bad_trees(bbm):
    from bbm_amd import _lib
    lib = _lib.load()
    m = bbm.fromString(THREE)
    desc, nd, _k = bbm.backbone.tree_desc(m)
    ws = torch.empty(1 << 16, dtype=torch.float64, device="cuda")
    sums = torch.empty(4, dtype=torch.float64, device="cuda")
    din, dout = _pairs(bbm, 256)
    probes = np.zeros((2, 7), np.float32)       # the tree takes 13 parameters
    rc = lib.bbm_hip_loss_tree(desc, nd, probes.ctypes.data, 7, 2, 256, din[0].data_ptr(), din[1].data_ptr(),
                               din[2].data_ptr(), dout[0].data_ptr(), dout[1].data_ptr(), dout[2].data_ptr(),
                               din[0].data_ptr(), din[1].data_ptr(), din[2].data_ptr(), 3, 3, 0, sums.data_ptr(),
                               ws.data_ptr(), ws.numel() * 8, None)
    assert rc == _lib.ERR_INVALID_ARG and b"13 parameters" in lib.bbm_hip_last_error()
