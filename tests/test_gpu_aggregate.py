"""aggregatemodel<MODELS...> of any models (include/bsdfmodel/aggregatemodel.h:22-222) on the GPU: the composed
path (bbm_hip_aggregate_*, bbm_amd.AggregateModel) against the reference's own variadic aggregates (golden
fixtures + 1M-pair batches from oracle/_ref), with the per-lane bar and proofs of tests/test_gpu_parity.py;
and the composed path against the fused Aggregate<Lambertian, X> kernels of the published fits' form."""
import numpy as np
import pytest

from tests import oracle_util as ou
from tests import test_gpu_parity as tp

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

META = ou.golden_meta()
INP = ou.golden_inputs()
COMPOSED = [k for k in META["models"] if k.startswith("Aggregate<") and k.count(",") >= 2 or
            k == "Aggregate<CookTorrance,GGX>"]


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd


def _composed(bbm, key, params):
    names = key[len("Aggregate<"):-1].split(",")
    kids, k = [], 0
    for nm in names:
        c = bbm.BsdfModel(nm)
        c.set_parameter_values(params[k:k + c._params.size])
        k += c._params.size
        kids.append(c)
    assert k == len(params)
    return bbm.Aggregate(*kids, fused=False)


def test_composed_keys_present():
    assert set(COMPOSED) == {"Aggregate<Lambertian,CookTorrance,GGX>", "Aggregate<CookTorrance,GGX>",
                             "Aggregate<OrenNayar,NganHe,Ward>"}


@pytest.mark.parametrize("key", COMPOSED)
def test_composed_aggregate_matches_reference_golden(bbm, key):
    g = ou.golden_model(key)
    stats = {}
    for si in range(len(META["models"][key]["sets"])):
        params = g[f"params{si}"]
        m = _composed(bbm, key, params)
        got = tp._gpu_evalpdf(m, INP["pin"], INP["pout"])
        prov = [tp._input_ulps_prover(lambda a, b: ou.oracle_eval_pdf(key, params, a, b, nthreads=8),
                                      [INP["pin"], INP["pout"]], got),
                tp._libm_prover(lambda a, b: ou.oracle_eval_pdf(key, params, a, b, nthreads=1),
                                [INP["pin"], INP["pout"]], got)]
        stats[f"{key}[{si}]"] = tp.check_lanes(got, g[f"evalpdf{si}"], f"{key}[{si}]", prov)
        refl = m.reflectance(tp._dev(INP["sout"])).cpu().numpy()
        tp.check_lanes(refl, g[f"reflectance{si}"], f"{key}[{si}] reflectance",
                       [tp._input_ulps_prover(lambda o: ou.ref_reflectance(key, params, o), [INP["sout"]], refl)])
        s = m.sample(tp._dev(INP["sout"]), tp._dev(INP["sxi"]))
        torch.cuda.synchronize()
        sg = np.concatenate([s.direction.cpu().numpy(), s.pdf.cpu().numpy()[None]], 0)
        sflag = s.flag.cpu().numpy()
        stats[f"{key}[{si}] sample"] = _check_composed_samples(key, params, INP["sout"], INP["sxi"], sg, sflag,
                                                                g[f"sample{si}"], g[f"sflag{si}"], f"{key}[{si}]")
    tp._report("aggregate_" + key.replace("<", "_").replace(">", "").replace(",", "_"), stats)


def _check_composed_samples(key, params, sout, sxi, got, flag, ref, ref_flag, what):
    """Flags identical; directions per lane (bar or proof); the sample's pdf = the reference's aggregate pdf at
    the GPU's direction (aggregatemodel.h:111-112 recomputes the mixture pdf there)."""
    assert np.array_equal(np.asarray(flag).astype(np.uint32), np.asarray(ref_flag).astype(np.uint32)), f"{what} flags"
    dok = tp._dir_ok(got[:3], ref[:3])
    bad = np.nonzero(~dok)[0]
    left = bad
    for prove in tp._sample_dir_provers(key, params, sout, sxi, got[:3]):
        if left.size == 0:
            break
        left = left[~prove(left)]
    assert left.size == 0, f"{what}: {left.size} sample directions outside 1e-5 and not proven, lanes {left[:4]}"
    pref = ou.oracle_eval_pdf(key, params, got[:3], sout, nthreads=8)[3]
    pref = np.where(np.asarray(ref_flag) == 0, ref[3], pref)
    return tp.check_lanes(got[3:], pref[None], f"{what} pdf(dir)",
                          [tp._input_ulps_prover(lambda a, b: ou.oracle_eval_pdf(key, params, a, b, nthreads=8)[3:],
                                                 [got[:3], sout], got[3:])])


@pytest.mark.parametrize("key", COMPOSED)
def test_composed_aggregate_large_batch(bbm, key):
    n = 1 << 20
    din = bbm.fill_directions(0xBB5EED, 0, 0, n, mode=0).cpu().numpy()
    dout = bbm.fill_directions(0xBB5EED, 1, 0, n, mode=1).cpu().numpy()
    params = ou.golden_model(key)["params0"]
    m = _composed(bbm, key, params)
    got = tp._gpu_evalpdf(m, din, dout)
    ref = ou.oracle_eval_pdf(key, params, din, dout, nthreads=8)
    tp.check_lanes(got, ref, f"{key} 1M", [tp._input_ulps_prover(
        lambda a, b: ou.oracle_eval_pdf(key, params, a, b, nthreads=8), [din, dout], got)])


def test_composed_equals_fused_for_the_fits_form(bbm):
    """Aggregate(Lambertian, X) through the fused kernel and through the composed path: the same per-lane
    results (the pdf division is the only rounding that may differ: fused div_nr vs the composed IEEE divide)."""
    n = 1 << 16
    din = bbm.fill_directions(7, 0, 0, n, mode=1)
    dout = bbm.fill_directions(7, 1, 0, n, mode=1)
    xi = torch.rand((2, n), generator=torch.Generator(device="cuda").manual_seed(9), device="cuda")
    for x in ("CookTorrance", "GGX", "NganHe", "Bagher"):
        lam, child = bbm.Lambertian(albedo=[0.2, 0.3, 0.4]), bbm.BsdfModel(x)
        fused = bbm.Aggregate(lam, child)
        composed = bbm.Aggregate(lam, child, fused=False)
        assert isinstance(fused, bbm.BsdfModel) and isinstance(composed, bbm.AggregateModel)
        fr, fp = fused.eval_pdf(din, dout)
        cr, cp = composed.eval_pdf(din, dout)
        torch.cuda.synchronize()
        assert torch.equal(fr, cr), x
        assert ou.parity_ok(cp.cpu().numpy(), fp.cpu().numpy()).all(), x
        fs, cs = fused.sample(dout, xi), composed.sample(dout, xi)
        torch.cuda.synchronize()
        assert torch.equal(fs.flag, cs.flag) and torch.equal(fs.direction, cs.direction), x
        assert ou.parity_ok(cs.pdf.cpu().numpy(), fs.pdf.cpu().numpy()).all(), x
        assert torch.equal(fused.reflectance(dout), composed.reflectance(dout)), x


def test_scratch_reuse_across_streams(bbm):
    """The stream-ordered scratch pool (bbm_hip.hip scratch_acquire / scratch_release): composed aggregates and
    He CDFs issued alternately on two streams, without host synchronisation between them, give exactly the
    results of the same calls issued one at a time (a block released on one stream and re-acquired on the other
    is waited for on the GPU)."""
    n = 1 << 18
    din = bbm.fill_directions(11, 0, 0, n, mode=1)
    dout = bbm.fill_directions(11, 1, 0, n, mode=1)
    torch.cuda.synchronize()
    models = [bbm.Aggregate(bbm.CookTorrance(), bbm.GGX(), fused=False),
              bbm.Aggregate(bbm.OrenNayar(), bbm.BsdfModel("NganHe"), bbm.Ward(), fused=False),
              bbm.BsdfModel("HeWestin")]
    want = []
    for m in models:
        rgb, pdf = m.eval_pdf(din, dout)
        torch.cuda.synchronize()
        want.append((rgb.clone(), pdf.clone(), m.reflectance(dout).clone()))
        torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    got = []
    for rep in range(3):
        for k, m in enumerate(models):
            s = streams[(rep + k) % 2]
            with torch.cuda.stream(s):
                rgb, pdf = m.eval_pdf(din, dout, stream=s)
                refl = m.reflectance(dout, stream=s)
            got.append((k, rgb, pdf, refl, s))
    torch.cuda.synchronize()
    for k, rgb, pdf, refl, _ in got:
        assert torch.equal(rgb, want[k][0]) and torch.equal(pdf, want[k][1]) and torch.equal(refl, want[k][2]), k


def test_scratch_held_by_captured_graph(bbm):
    """A HIP graph that captured library calls using scratch (a composed aggregate's per-lane terms, He's sampler
    CDF) keeps those blocks: the pool pins them at capture, so scratch_trim and later uncaptured calls -- which
    would otherwise free or reuse them -- leave the graph's replays correct."""
    n = 1 << 16
    din = bbm.fill_directions(13, 0, 0, n, mode=1)
    dout = bbm.fill_directions(13, 1, 0, n, mode=1)
    models = [bbm.Aggregate(bbm.CookTorrance(), bbm.GGX(), bbm.Lambertian(), fused=False), bbm.BsdfModel("HeWestin")]
    want, outs = [], []
    for m in models:
        rgb, pdf = m.eval_pdf(din, dout)
        torch.cuda.synchronize()
        want.append((rgb.clone(), pdf.clone()))
        outs.append((torch.empty_like(rgb), torch.empty_like(pdf)))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for m, (r, p) in zip(models, outs):
            m.eval_pdf(din, dout, rgb=r, pdf=p, stream=side)
    torch.cuda.synchronize()
    held = bbm.scratch_bytes()
    bbm.scratch_trim()
    assert bbm.scratch_bytes() > 0 and bbm.scratch_bytes() <= held
    # uncaptured calls of other sizes in between: they must not be handed the graph's blocks
    for m in models:
        m.eval_pdf(dout[:, : n // 2], din[:, : n // 2])
    for _ in range(2):
        for r, p in outs:
            r.zero_()
            p.zero_()
        g.replay()
        torch.cuda.synchronize()
        for (r, p), (wr, wp) in zip(outs, want):
            assert torch.equal(r, wr) and torch.equal(p, wp)
    del g
    torch.cuda.synchronize()
    bbm.scratch_trim_captured()


def test_scratch_bounded_over_repeated_captures(bbm):
    """Capture, replay, destroy and trim (bbm_hip_scratch_trim_captured) N times: the scratch a capture pins is
    released with its graph, so the pool does not grow with the number of captures."""
    n = 1 << 14
    din = bbm.fill_directions(21, 0, 0, n, mode=1)
    dout = bbm.fill_directions(21, 1, 0, n, mode=1)
    m = bbm.Aggregate(bbm.CookTorrance(), bbm.GGX(), bbm.Lambertian(), fused=False)
    rgb, pdf = torch.empty((3, n), device="cuda"), torch.empty(n, device="cuda")
    sizes = []
    for _ in range(6):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            m.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=side)
        g.replay()
        torch.cuda.synchronize()
        del g
        torch.cuda.synchronize()
        bbm.scratch_trim_captured()
        bbm.scratch_trim()
        sizes.append(bbm.scratch_bytes())
    assert max(sizes) == min(sizes), f"scratch grew over captures: {sizes}"
