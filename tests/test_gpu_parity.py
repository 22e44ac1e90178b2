"""Parity of the HIP backbone with the reference (GPU; run with -m gpu on an MI355X).

Every check goes through the C-ABI (libbbm_hip via bbm_amd) and is compared with
  * the reference's own outputs (tests/golden, floatRGB, written by oracle/gen_golden.py), and
  * the reference itself (oracle/_ref, prebuilt) on fresh seeded batches of 1M pairs.

The bar (BASELINE.json north_star: <= 1e-5 relative) is applied lane by lane, with no batch-dependent floor
(tests/oracle_util.parity_ok): |gpu - ref| <= 1e-5 |ref| for every normal reference value, the same absolute
step (1e-5 FLT_MIN) below the normal range, NaN for NaN.  A lane outside the bar fails unless it is proven on
its own, by one of three per-lane arguments, and the number of such lanes is reported and bounded:
  * input ulps (backward error): the reference itself, at inputs moved by <= 2 float steps per coordinate,
    produces values on both sides of the GPU's (oracle_util.explained_by_input_ulps) -- the lane's difference
    is the reference's own sensitivity to the last bits of its input (subnormal intermediates, cancellation);
  * libm last bit: the reference itself reproduces the GPU value when one call of one glibc float function
    (erff, expf, sinf, ...) returns its neighbouring float (oracle/libm_ulp.c; glibc's erff / erfcf are not
    correctly rounded on ~6 % of inputs, and an inverse-CDF sample at a clamped xi hinges on that bit);
  * sampler CDF (the data-driven samplers of the He family): the GPU pdf is what the reference's pdf
    arithmetic gives on the CDF built from the GPU's backscatter evaluations, and those evaluations meet the
    bar (oracle_util.sampler_cdf / sampler_pdf): a 1-ulp difference in one of the 90 evaluations moves the
    pdf of the neighbouring bins by up to ~2e-5 through the CDF's differences.
"""
import json
import os

import numpy as np
import pytest

from tests import oracle_util as ou

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

META = ou.golden_meta()
INP = ou.golden_inputs()
TABULATED_SAMPLERS = {"He", "HeWestin", "HeHolzschuch", "NganHe"}
MAX_EXCUSED_FRAC = 1e-3       # at most this fraction of a batch's lanes may need an input-ulps proof
# ... a sampler-CDF proof (a CDF entry moves the ~2/90 of directions in its bins).  Round 5: none may -- the He family's
# 90 backscatter evaluations behind the CDF follow the reference's float complex Fresnel (he.hpp FresnelComplexRGB),
# within 1-4 ulp where not bit-identical, and no lane of any golden set or 1 M batch needed this proof (r05_parity_*.json;
# round 4: 6 509 eval/pdf and 1 279 sampling lanes per 1 M for HeWestin).  The prover stays as the diagnostic.
MAX_SAMPLER_FRAC = 0.0
# Ceiling on the relative error of the lanes that pass by a proof (the proofs bound WHY a lane differs, this bounds
# HOW MUCH).  History: round 3 Bagher / Aggregate(Lambertian, Bagher) 5e-2 and the He family 2e-2 (the ill-conditioned
# lanes of Bagher's shadowing 1 + Lambda (1 - e^(c t^k)) and of He's series at tiny D); round 4 (glibc powf / expf /
# logf / erfcf restated) Bagher 5e-3, Aggregate(Lambertian, Bagher) 2e-2, the rest 1e-3.  Round 5 (Bagher's D by
# glibc's powf / expf in every mode): Aggregate(Lambertian, Bagher) bit-identical on both 1M-pair batches, no proven
# lane of any model at or above TINY off by more than 1.7e-5 (HeWestin; profiles/r05_parity_*.json) -- one ceiling
# for all.  Below TINY the default mode rounds quotients of subnormal intermediates on the normal grid
# (set_exact_subnormals), and Bagher's proven lanes there reach 5.3e-3 on values ~1e-36: TINY_REL_CEILING.
EXCUSED_REL_CEILING = {}
EXCUSED_REL_DEFAULT = 1e-4
TINY = 1e-30
TINY_REL_CEILING = 1e-2


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def _gpu_evalpdf(model, din, dout, **kw):
    rgb, pdf = model.eval_pdf(_dev(din), _dev(dout), **kw)
    torch.cuda.synchronize()
    return np.concatenate([rgb.cpu().numpy(), pdf.cpu().numpy()[None]], 0)


def _save(tag, arr):
    d = os.path.join(ou.ROOT, "gpurun_out", "gpu_outputs")
    os.makedirs(d, exist_ok=True)
    np.save(os.path.join(d, tag + ".npy"), arr)


def _report(tag, stats):
    os.makedirs(os.path.join(ou.ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ou.ROOT, "gpurun_out", f"parity_{tag}.json"), "w") as f:
        json.dump(stats, f, indent=1)
    for k, v in stats.items():
        print(f"{tag} {k}: {v}")


def check_lanes(got, ref, what, provers=(), model=None):
    """Apply the per-lane bar to (channels, lanes) arrays; lanes outside it must be proven by one of `provers`
    (functions lanes -> bool array), and even a proven lane must stay within the model's EXCUSED_REL_CEILING
    (`model`, default: the name `what` starts with); returns the statistics reported under gpurun_out/parity_*.json."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    n = got.shape[-1]
    ok = ou.parity_ok(got, ref).reshape(-1, n).all(0)
    bad = np.nonzero(~ok)[0]
    proven = {}
    left = bad
    for prove in provers:
        if left.size == 0:
            break
        p = np.asarray(prove(left), bool)
        proven[prove.__name__] = int(p.sum())
        left = left[~p]
    if left.size:
        i = left[:4]
        raise AssertionError(f"{what}: {left.size} of {n} lanes outside the 1e-5 bar and not proven; lanes {i}: "
                             f"got {got[..., i].T.tolist()} ref {ref[..., i].T.tolist()}")
    n_sampler = proven.get("sampler_cdf", 0)
    assert bad.size - n_sampler <= max(2, MAX_EXCUSED_FRAC * n), \
        f"{what}: {bad.size - n_sampler} of {n} lanes needed an input-ulps proof ({proven})"
    assert n_sampler <= MAX_SAMPLER_FRAC * n, f"{what}: {n_sampler} of {n} lanes needed a sampler-CDF proof"
    gb, rb = got[..., bad], ref[..., bad]
    big = np.abs(rb) >= TINY
    excused = ou.max_rel_normal(np.where(big, gb, rb), rb) if bad.size else 0.0
    excused_tiny = ou.max_rel_normal(np.where(big, rb, gb), rb) if bad.size else 0.0
    ceiling = EXCUSED_REL_CEILING.get(model or what.split("[")[0].split(" ")[0].split("/")[0], EXCUSED_REL_DEFAULT)
    assert excused <= ceiling, f"{what}: a proven lane is {excused:.3e} off (ceiling {ceiling:g})"
    assert excused_tiny <= TINY_REL_CEILING, \
        f"{what}: a proven lane below {TINY:g} is {excused_tiny:.3e} off (ceiling {TINY_REL_CEILING:g})"
    sub = (np.abs(ref) < ou.FLT_MIN) & (ref != 0)
    return {"lanes": int(n), "max_rel_normal": ou.max_rel_normal(got, ref), "max_rel_proven": excused,
            "max_rel_proven_below_tiny": excused_tiny,
            "max_ulp": int(ou.ulp_diff(got, ref).max()) if got.size else 0,
            "frac_bit_exact": float(np.mean(ou.ulp_diff(got, ref) == 0)) if got.size else 1.0,
            "subnormal_ref_values": int(sub.sum()), "lanes_outside_bar": int(bad.size),
            "proven_by": proven}


def _input_ulps_prover(ref_fn, inputs, got, any_match=False, abs_tol=0.0):
    """Prover: the backward-error argument over the given lanes of `inputs` (list of (k, n) arrays): inputs moved
    by <= 2 float steps per coordinate, then (for the lanes still unproven) <= 4."""
    def input_ulps(lanes):
        ok = ou.explained_by_input_ulps(ref_fn, [a[:, lanes] for a in inputs], got[:, lanes], k=2,
                                        any_match=any_match, abs_tol=abs_tol)
        rest = lanes[~ok]
        if rest.size:
            ok[~ok] = ou.explained_by_input_ulps(ref_fn, [a[:, rest] for a in inputs], got[:, rest], k=4,
                                                 trials=128, any_match=any_match, abs_tol=abs_tol)
        return ok
    return input_ulps


def _libm_prover(ref_fn, inputs, got, any_match=False, abs_tol=0.0):
    """Prover: one glibc float call moved by one ulp (oracle/libm_ulp.c) reproduces the GPU value; ref_fn must
    evaluate in the calling thread (nthreads=1)."""
    def libm_ulp(lanes):
        return ou.explained_by_libm_ulp(ref_fn, [a[:, lanes] for a in inputs], got[:, lanes], any_match=any_match,
                                        abs_tol=abs_tol)
    return libm_ulp


def _sampler_prover(bbm, name, params, din, dout, pdf_got, eval_got=None, component=3, unit=0):
    """Prover for the tabulated samplers' pdf: see the module docstring.  pdf_got: (n,) GPU pdfs of the pairs
    (din, dout); eval_got: their (3, n) eval channels, which must meet the bar for a lane to be proven here."""
    hb = ou.sampler_backscatter_dirs()
    p = np.asarray(params, np.float32).copy()
    if name == "NganHe":
        p[:3] = 1.0          # scaledmodel wraps the sampler from outside: the CDF sees the unscaled he_base
    m = bbm.BsdfModel(name)
    m.set_parameter_values(p)
    gpu_bs = _gpu_evalpdf(m, hb, hb, component=bbm.bsdf_flag(component), unit=bbm.unit_t(unit))
    ref_bs = ou.oracle_eval_pdf(name, p, hb, hb, component, unit, nthreads=8)

    def sampler_cdf(lanes):
        if not ou.parity_ok(gpu_bs[:3], ref_bs[:3]).all():
            return np.zeros(lanes.size, bool)
        want = ou.sampler_pdf(ou.sampler_cdf(gpu_bs[:3]), din[:, lanes], dout[:, lanes])
        ok = ou.parity_ok(pdf_got[lanes], want)
        if eval_got is not None:
            ok &= ou.parity_ok(eval_got[:, lanes], ou.oracle_eval_pdf(name, params, din[:, lanes], dout[:, lanes],
                                                                      component, unit, nthreads=8)[:3]).all(0)
        return ok
    return sampler_cdf


def _evalpdf_provers(bbm, name, params, din, dout, got, component=3, unit=0):
    provers = []
    if name in TABULATED_SAMPLERS:    # first: a pdf moved by a CDF entry is explained by the CDF, not the input
        provers.append(_sampler_prover(bbm, name, params, din, dout, got[3], got[:3], component, unit))
    provers.append(_input_ulps_prover(lambda a, b: ou.oracle_eval_pdf(name, params, a, b, component, unit, nthreads=8),
                                      [din, dout], got))
    provers.append(_libm_prover(lambda a, b: ou.oracle_eval_pdf(name, params, a, b, component, unit, nthreads=1),
                                [din, dout], got))
    return provers


def _gpu_models(bbm):
    return [m for m in bbm.model_names() if m in META["models"]]


def test_every_gpu_model_matches_reference_golden(bbm):
    stats = {}
    for name in _gpu_models(bbm):
        g = ou.golden_model(name)
        for si in range(len(META["models"][name]["sets"])):
            params = g[f"params{si}"]
            m = bbm.BsdfModel(name)
            m.set_parameter_values(params)
            got = _gpu_evalpdf(m, INP["pin"], INP["pout"])
            _save(f"golden_{name}_{si}", got)
            stats[f"{name}[{si}]"] = check_lanes(got, g[f"evalpdf{si}"], f"{name}[{si}]",
                                                 _evalpdf_provers(bbm, name, params, INP["pin"], INP["pout"], got))
    _report("golden", stats)


def test_reflectance_matches_reference_golden(bbm):
    """reflectance(out) (concepts/bsdfmodel.h: Spectrum reflectance(out, component, unit, mask)) for
    every parameter set and per component; it is also the sampling weight of Aggregate models."""
    stats = {}
    for name in _gpu_models(bbm):
        g = ou.golden_model(name)
        for si in range(len(META["models"][name]["sets"])):
            params = g[f"params{si}"]
            m = bbm.BsdfModel(name)
            m.set_parameter_values(params)
            got = m.reflectance(_dev(INP["sout"])).cpu().numpy()
            prove = _input_ulps_prover(lambda o, p=params: ou.ref_reflectance(name, p, o), [INP["sout"]], got)
            stats[f"{name}[{si}]"] = check_lanes(got, g[f"reflectance{si}"], f"{name}[{si}] reflectance", [prove])
        m = bbm.BsdfModel(name)
        m.set_parameter_values(g["params0"])
        for tag, comp in (("diffuse", 1), ("specular", 2)):
            got = m.reflectance(_dev(INP["sout"]), component=bbm.bsdf_flag(comp)).cpu().numpy()
            prove = _input_ulps_prover(lambda o, c=comp: ou.ref_reflectance(name, g["params0"], o, c), [INP["sout"]], got)
            check_lanes(got, g[f"reflectance_{tag}"], f"{name}/{tag} reflectance", [prove])
    _report("reflectance", stats)


@pytest.mark.parametrize("tag,comp,unit", [("diffuse", 1, 0), ("specular", 2, 0), ("importance", 3, 1)])
def test_component_and_unit_semantics(bbm, tag, comp, unit):
    for name in _gpu_models(bbm):
        g = ou.golden_model(name)
        m = bbm.BsdfModel(name)
        m.set_parameter_values(g["params0"])
        got = _gpu_evalpdf(m, INP["pin"], INP["pout"], component=bbm.bsdf_flag(comp), unit=bbm.unit_t(unit))
        check_lanes(got, g[f"evalpdf_{tag}"], f"{name}/{tag}",
                    _evalpdf_provers(bbm, name, g["params0"], INP["pin"], INP["pout"], got, comp, unit))


def test_eval_pdf_fused_equals_separate_calls(bbm):
    n = 100_003   # odd size: vector body + scalar tail
    din = bbm.fill_directions(11, 0, 0, n, mode=1)
    dout = bbm.fill_directions(11, 1, 0, n, mode=1)
    for name in _gpu_models(bbm):
        m = bbm.BsdfModel(name)
        rgb, pdf = m.eval_pdf(din, dout)
        rgb2 = m.eval(din, dout)
        pdf2 = m.pdf(din, dout)
        torch.cuda.synchronize()
        assert torch.equal(rgb, rgb2) and torch.equal(pdf, pdf2), name


@pytest.mark.parametrize("mode_in,mode_out", [(0, 1), (0, 0)])
def test_large_batch_vs_reference(bbm, mode_in, mode_out):
    """1M pairs per model and parameter set against the reference itself (prebuilt oracle/_ref shim): upper
    hemisphere in with sphere out (~50 % masked lanes) and both on the upper hemisphere (every lane active)."""
    n = 1 << 20
    din = bbm.fill_directions(0xBB5EED, 0, 0, n, mode=mode_in).cpu().numpy()
    dout = bbm.fill_directions(0xBB5EED, 1, 0, n, mode=mode_out).cpu().numpy()
    stats = {}
    for name in _gpu_models(bbm):
        if name not in ou.oracle_models():
            continue
        g = ou.golden_model(name)
        for si in range(len(META["models"][name]["sets"])):
            params = g[f"params{si}"]
            m = bbm.BsdfModel(name)
            m.set_parameter_values(params)
            got = _gpu_evalpdf(m, din, dout)
            ref = ou.oracle_eval_pdf(name, params, din, dout, nthreads=8)
            stats[f"{name}[{si}]"] = check_lanes(got, ref, f"{name}[{si}] {mode_in}{mode_out}",
                                                 _evalpdf_provers(bbm, name, params, din, dout, got))
    _report(f"large_{mode_in}{mode_out}", stats)
    # beyond the bar: the models that return the reference's floats on every lane stay that way (DESIGN §4.2 table;
    # round 6 added the Ward family)
    for key, st in stats.items():
        if key.split("[")[0] in BIT_IDENTICAL:
            assert st["frac_bit_exact"] == 1.0, f"{key} {mode_in}{mode_out}: {st['frac_bit_exact']} bit-identical"


BIT_IDENTICAL = {
    "Lambertian", "GGX", "GGXHeitz", "OrenNayar", "Phong", "NganBlinnPhong", "Lafortune", "NganLafortune", "LowSmooth",
    "Ward", "WardDuer", "WardDuerGeislerMoroder", "NganWard", "NganWardDuer",
    "Aggregate<Lambertian,Bagher>", "Aggregate<Lambertian,CookTorrance>", "Aggregate<Lambertian,GGX>",
    "Aggregate<Lambertian,LowAshikhminShirley>", "Aggregate<Lambertian,LowCookTorrance>", "Aggregate<Lambertian,LowSmooth>",
    "Aggregate<Lambertian,NganAshikhminShirley>", "Aggregate<Lambertian,NganBlinnPhong>",
    "Aggregate<Lambertian,NganCookTorrance>", "Aggregate<Lambertian,NganHe>", "Aggregate<Lambertian,NganLafortune>",
    "Aggregate<Lambertian,NganWard>", "Aggregate<Lambertian,NganWardDuer>"}


EXACT_MODELS = ("CookTorrance", "CookTorranceWalter", "CookTorranceHeitz", "NganCookTorrance")


@pytest.mark.parametrize("mode_in,mode_out", [(0, 1), (0, 0)])
def test_exact_subnormal_mode_is_bit_exact(bbm, mode_in, mode_out):
    """bbm_hip_set_exact_subnormals(1): the Beckmann microfacet models' eval + pdf equal the reference's floats on
    every lane of 1M pairs per parameter set (the quotients reached by subnormal intermediates rounded as glibc's
    IEEE divisions; bit-exact fraction >= 0.9999), and differ from the default mode only on values below 1e-30.
    Unaligned sizes take the scalar kernel's exact instantiation."""
    n = 1 << 20
    din = bbm.fill_directions(0xBB5EED, 0, 0, n, mode=mode_in).cpu().numpy()
    dout = bbm.fill_directions(0xBB5EED, 1, 0, n, mode=mode_out).cpu().numpy()
    stats = {}
    try:
        for name in EXACT_MODELS:
            g = ou.golden_model(name)
            for si in range(len(META["models"][name]["sets"])):
                params = g[f"params{si}"]
                m = bbm.BsdfModel(name)
                m.set_parameter_values(params)
                assert bbm.set_exact_subnormals(False) in (False, True)
                fast = _gpu_evalpdf(m, din, dout)
                assert bbm.set_exact_subnormals(True) is False
                got = _gpu_evalpdf(m, din, dout)
                # scalar kernel: row views starting one float in (4 B-aligned pointers)
                di, do = torch.from_numpy(din).cuda(), torch.from_numpy(dout).cuda()
                o_rgb, o_pdf = m.eval_pdf(tuple(di[i, 1:n - 2] for i in range(3)), tuple(do[i, 1:n - 2] for i in range(3)))
                odd = torch.cat([o_rgb, o_pdf[None]]).cpu().numpy()
                ref = ou.oracle_eval_pdf(name, params, din, dout, nthreads=8)
                s = check_lanes(got, ref, f"exact {name}[{si}] {mode_in}{mode_out}",
                                _evalpdf_provers(bbm, name, params, din, dout, got))
                assert s["frac_bit_exact"] >= 0.9999, f"exact {name}[{si}]: {s}"
                assert np.array_equal(odd, got[:, 1:n - 2], equal_nan=True), f"exact {name}[{si}]: scalar kernel differs"
                diff = ~((fast == got) | (np.isnan(fast) & np.isnan(got)))
                s["max_ref_where_modes_differ"] = float(np.abs(ref[diff]).max()) if diff.any() else 0.0
                assert s["max_ref_where_modes_differ"] < 1e-30, f"exact {name}[{si}]: modes differ above 1e-30 ({s})"
                s["frac_bit_exact_default_mode"] = float(np.mean(ou.ulp_diff(fast, ref) == 0))
                stats[f"{name}[{si}]"] = s
    finally:
        bbm.set_exact_subnormals(False)
    _report(f"exact_{mode_in}{mode_out}", stats)


# exact mode beyond the Beckmann quotients: model -> bit-identical fraction it must reach on every parameter set
EXACT_MODE_FLOOR = {"Bagher": 0.999, "Aggregate<Lambertian,Bagher>": 0.999, "LowMicrofacet": 0.999,
                    "LowMicrofacetFit": 0.999, "Ribardiere": 0.0, "LowSmooth": 0.999}


@pytest.mark.parametrize("name", list(EXACT_MODE_FLOOR))
def test_exact_mode_models(bbm, name):
    """Exact mode for the NDFs whose default evaluation approximates a power: Bagher's D by glibc's powf / expf
    (spectral.hpp eval_geo<true>; with the glibc shadowing term and theta already exact), the Low and Student-T
    NDFs' double pow by f64::pow_d rounded to float.  Bagher and the Low microfacet models are then the reference's
    floats on nearly every lane of 1M hemisphere pairs per parameter set (the default mode's fast powers leave
    52-93 %); Ribardiere's Student-T shadowing keeps its f32 fits (more bit-identical lanes, not all).  0 lanes outside
    the bar either way."""
    n = 1 << 20
    din = bbm.fill_directions(0xBB5EED, 0, 0, n, mode=0).cpu().numpy()
    dout = bbm.fill_directions(0xBB5EED, 1, 0, n, mode=0).cpu().numpy()
    stats = {}
    try:
        g = ou.golden_model(name)
        for si in range(len(META["models"][name]["sets"])):
            params = g[f"params{si}"]
            m = bbm.BsdfModel(name)
            m.set_parameter_values(params)
            bbm.set_exact_subnormals(True)
            got = _gpu_evalpdf(m, din, dout)
            bbm.set_exact_subnormals(False)
            fast = _gpu_evalpdf(m, din, dout)
            ref = ou.oracle_eval_pdf(name, params, din, dout, nthreads=8)
            s = check_lanes(got, ref, f"exact {name}[{si}]", _evalpdf_provers(bbm, name, params, din, dout, got))
            s["frac_bit_exact_default_mode"] = float(np.mean(ou.ulp_diff(fast, ref) == 0))
            assert s["frac_bit_exact"] >= EXACT_MODE_FLOOR[name], f"exact {name}[{si}]: {s}"
            assert s["frac_bit_exact"] >= s["frac_bit_exact_default_mode"], s
            stats[f"{name}[{si}]"] = s
    finally:
        bbm.set_exact_subnormals(False)
    _report(f"exact_{name.replace('<', '_').replace(',', '_').replace('>', '')}", stats)


def test_mask_lanes_are_zero_and_others_untouched(bbm):
    n = 4099
    din = bbm.fill_directions(3, 0, 0, n, mode=0)
    dout = bbm.fill_directions(3, 1, 0, n, mode=0)
    mask = (torch.arange(n, device="cuda") % 3 != 0)
    for name in _gpu_models(bbm):
        m = bbm.BsdfModel(name)
        rgb, pdf = m.eval_pdf(din, dout)
        rgbm, pdfm = m.eval_pdf(din, dout, mask=mask)
        torch.cuda.synchronize()
        assert torch.equal(rgbm[:, mask], rgb[:, mask]) and torch.equal(pdfm[mask], pdf[mask])
        assert (rgbm[:, ~mask] == 0).all() and (pdfm[~mask] == 0).all()


def test_unaligned_and_tiny_sizes(bbm):
    """Scalar path (unaligned views) and n = 0..9 give the same results as the vector path."""
    n = 1000
    din = bbm.fill_directions(5, 0, 0, n + 1, mode=1)
    dout = bbm.fill_directions(5, 1, 0, n + 1, mode=1)
    m = bbm.CookTorrance()
    a_rgb, a_pdf = m.eval_pdf(din[:, 1:].contiguous(), dout[:, 1:].contiguous())
    u_rgb, u_pdf = m.eval_pdf(tuple(din[i, 1:] for i in range(3)), tuple(dout[i, 1:] for i in range(3)))
    torch.cuda.synchronize()
    assert torch.equal(a_rgb, u_rgb) and torch.equal(a_pdf, u_pdf)
    f_rgb, f_pdf = m.eval_pdf(din[:, :n].contiguous(), dout[:, :n].contiguous())
    for k in range(10):
        rgb, pdf = m.eval_pdf(din[:, :k].contiguous(), dout[:, :k].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(rgb, f_rgb[:, :k]) and torch.equal(pdf, f_pdf[:k])


def test_fill_directions_shards_regenerate_global_batch(bbm):
    full = bbm.fill_directions(42, 0, 0, 10_000, mode=1)
    part = bbm.fill_directions(42, 0, 6_000, 4_000, mode=1)
    torch.cuda.synchronize()
    assert torch.equal(full[:, 6000:], part)
    ref = ou.dirgen_numpy(42, 0, 0, 10_000, mode=1)
    np.testing.assert_allclose(full.cpu().numpy(), ref, atol=2e-6)


def test_errors_raise(bbm):
    m = bbm.CookTorrance()
    d = bbm.fill_directions(1, 0, 0, 16)
    with pytest.raises(ValueError):
        m.eval_pdf(d, d[:, :8].contiguous())
    with pytest.raises(TypeError):
        m.eval_pdf(d.double(), d)
    # caller-supplied outputs are validated before the launch (an undersized or foreign buffer would be written
    # out of bounds by the kernel)
    with pytest.raises(ValueError):
        m.eval_pdf(d, d, rgb=torch.empty((3, 8), device="cuda"))
    with pytest.raises(ValueError):
        m.eval_pdf(d, d, pdf=torch.empty((15,), device="cuda"))
    with pytest.raises(TypeError):
        m.eval_pdf(d, d, rgb=torch.empty((3, 16), dtype=torch.float64, device="cuda"))
    with pytest.raises(ValueError):
        m.eval_pdf(d, d, rgb=torch.empty((16, 3), device="cuda").t())


# ----------------------------------------------------------------------------------------------- sampling
#
# Directions are unit vectors: a sample's direction meets the bar where every component is within 1e-5 of the
# reference's (1e-5 of the vector's length).  A lane outside it must be proven, like an eval lane, by the
# reference at inputs (out, xi) moved by <= 2 float steps; for the tabulated samplers also by a CDF bin flip:
# the sampled bin's within-bin warp is discontinuous at the bin edges (ndf/sampler.h:63-92, util/cdf.h:73-83)
# and a 1-ulp CDF difference moves an xi0 that close to an edge into the neighbouring bin, so such a lane
# passes when the reference, given an xi0 at most FLIP_ULPS float steps away, returns the GPU's direction
# (to FLIP_DIR_TOL: the warp is steep there).  Flags must be identical, and the pdf of a sample is checked
# with the eval bar against the reference's pdf at the GPU's own direction.
DIR_TOL = 1e-5
FLIP_ULPS = 1024
FLIP_DIR_TOL = 1e-4


def _dir_ok(got, ref):
    with np.errstate(invalid="ignore"):
        return ((np.abs(np.asarray(got, np.float64) - ref) <= DIR_TOL) |
                (np.isnan(got) & np.isnan(ref))).all(0)


def _sample_dir_provers(name, params, dout, xi, got_dir, component=3):
    def ref_dirs(o, x):
        d, _ = ou.oracle_sample(name, params, o, x, component=component, nthreads=8)
        return d[:3]
    input_ulps = _input_ulps_prover(ref_dirs, [dout, xi], got_dir, any_match=True, abs_tol=DIR_TOL)
    libm_ulp = _libm_prover(lambda o, x: ou.oracle_sample(name, params, o, x, component=component, nthreads=1)[0][:3],
                            [dout, xi], got_dir, any_match=True, abs_tol=DIR_TOL)

    def cdf_bin_flip(lanes):
        if name not in TABULATED_SAMPLERS:
            return np.zeros(lanes.size, bool)
        x0 = xi[0, lanes].astype(np.float32)
        steps = np.concatenate([-np.arange(1, FLIP_ULPS + 1), np.arange(1, FLIP_ULPS + 1)])
        xs = ou.perturb_ulps(np.repeat(x0[:, None], steps.size, 1), np.broadcast_to(steps, (x0.size, steps.size)))
        xs = np.clip(xs, 0, 1).astype(np.float32)
        m = steps.size
        o = np.ascontiguousarray(np.repeat(dout[:, lanes], m, axis=1))
        x = np.ascontiguousarray(np.stack([xs.ravel(), np.repeat(xi[1, lanes], m)]).astype(np.float32))
        ref, _ = ou.oracle_sample(name, params, o, x, component=component, nthreads=8)
        d = np.abs(np.repeat(got_dir[:, lanes], m, axis=1) - ref[:3]).max(0).reshape(lanes.size, m)
        return np.nanmin(d, axis=1) <= FLIP_DIR_TOL
    return [input_ulps, libm_ulp, cdf_bin_flip]


def _pdf_at_dir(name, params, dirs, outs, xi, flags):
    """The pdf the reference's sampler would report for a sample at `dirs`.  For every model but
    one that is pdf(dir, out).  AshikhminShirleyFull's one-sample mixture
    (ashikhminshirleyfull.h:96-124) draws a specular candidate with xi0 / w_s and a diffuse one
    with (xi0 - w_s) / w_d (0 when w_d <= eps), returns the one selected by xi0 <= w_s, and
    reports w_s pdf_s(specular candidate) + w_d pdf_d(diffuse candidate): the chosen candidate's
    pdf is taken at the GPU direction, the other candidate is drawn by the reference itself."""
    if name != "AshikhminShirleyFull":
        return ou.oracle_eval_pdf(name, params, dirs, outs, nthreads=8)[3]
    p = np.asarray(params, np.float32)
    one, eps = np.float32(1), np.finfo(np.float32).eps
    spec_albedo = (p[3] + p[4]) + p[5]
    diff_albedo = ((p[0] + p[1]) + p[2]) * (one - spec_albedo)
    dw = diff_albedo / (diff_albedo + spec_albedo)
    sw = one - dw
    xi = np.asarray(xi, np.float32)
    xs = np.stack([xi[0] / sw if sw > eps else np.zeros_like(xi[0]), xi[1]])
    xd = np.stack([(xi[0] - sw) / dw if dw > eps else np.zeros_like(xi[0]), xi[1]])
    flags = np.asarray(flags)
    ps = np.where(flags == 2, ou.oracle_eval_pdf(name, params, dirs, outs, component=2, nthreads=8)[3],
                  ou.oracle_sample(name, params, outs, xs, component=2, nthreads=8)[0][3])
    pd = np.where(flags == 1, ou.oracle_eval_pdf(name, params, dirs, outs, component=1, nthreads=8)[3],
                  ou.oracle_sample(name, params, outs, xd, component=1, nthreads=8)[0][3])
    return (sw * ps.astype(np.float32) + dw * pd.astype(np.float32)).astype(np.float32)


def _check_samples(bbm, name, params, sout, sxi, got, flag, ref, ref_flag, what):
    """Flags identical; directions per lane (bar or proof); sample pdf vs the reference pdf at the GPU's
    direction (the reference's own sample pdf on rejected lanes, whose all-zero direction has no pdf)."""
    assert np.array_equal(np.asarray(flag).astype(np.uint32), np.asarray(ref_flag).astype(np.uint32)), f"{what} flags"
    dok = _dir_ok(got[:3], ref[:3])
    bad = np.nonzero(~dok)[0]
    proven = {}
    left = bad
    for prove in _sample_dir_provers(name, params, sout, sxi, got[:3]):
        if left.size == 0:
            break
        p = prove(left)
        proven[prove.__name__] = int(p.sum())
        left = left[~p]
    assert left.size == 0, (f"{what}: {left.size} sample directions outside 1e-5 and not proven, lanes {left[:4]}: "
                            f"got {got[:3, left[:4]].T.tolist()} ref {ref[:3, left[:4]].T.tolist()}")
    # the golden set's 690 samples include 33 deliberately ill-conditioned edge cases (xi on the clamps,
    # grazing views), hence the floor of 8
    assert bad.size <= max(8, MAX_EXCUSED_FRAC * dok.size), f"{what}: {bad.size} directions needed a proof"
    rejected = np.asarray(ref_flag) == 0
    pref = np.where(rejected, ref[3], _pdf_at_dir(name, params, got[:3], sout, sxi, flag))
    provers = []
    if name in TABULATED_SAMPLERS:
        provers.append(_sampler_prover(bbm, name, params, got[:3], sout, got[3]))
    if name != "AshikhminShirleyFull":
        provers.append(_input_ulps_prover(lambda a, b: ou.oracle_eval_pdf(name, params, a, b, nthreads=8)[3:],
                                          [got[:3], sout], got[3:]))
        provers.append(_libm_prover(lambda a, b: ou.oracle_eval_pdf(name, params, a, b, nthreads=1)[3:],
                                    [got[:3], sout], got[3:]))
    else:
        # the one-sample mixture's pdf (w_s pdf_s + w_d pdf_d, either weight may be negative for out-of-range
        # albedos, so it can cancel): the same input-ulps argument over (direction, out, xi) and its flag
        def mixture_input_ulps(lanes):
            ok = np.zeros(lanes.size, bool)
            for k, trials in ((2, 48), (4, 128)):
                rest = ~ok
                if not rest.any():
                    break
                sub = lanes[rest]
                fl = np.tile(np.asarray(flag)[sub], trials)     # moved inputs come trial by trial
                ok[rest] = ou.explained_by_input_ulps(lambda d, o, x: _pdf_at_dir(name, params, d, o, x, fl)[None],
                                                      [got[:3, sub], sout[:, sub], sxi[:, sub]], got[3:, sub], k=k,
                                                      trials=trials)
            return ok
        provers.append(mixture_input_ulps)
    st = check_lanes(got[3:], pref[None], f"{what} pdf(dir)", provers)
    st["max_dir_abs_err"] = float(np.nanmax(np.abs(got[:3].astype(np.float64) - ref[:3]))) if got.size else 0.0
    st["frac_dir_within_1e-6"] = float(np.mean(np.abs(got[:3].astype(np.float64) - ref[:3]).max(0) <= 1e-6))
    st["dir_lanes_outside_bar"] = int(bad.size)
    st["dir_proven_by"] = proven
    return st


def _gpu_sample(model, sout, sxi, **kw):
    s = model.sample(_dev(sout), _dev(sxi), **kw)
    torch.cuda.synchronize()
    return np.concatenate([s.direction.cpu().numpy(), s.pdf.cpu().numpy()[None]], 0), s.flag.cpu().numpy()


def test_sample_matches_reference_golden(bbm):
    """sample(out, xi) -> (direction, pdf, flag) vs the reference's own samples (golden)."""
    stats = {}
    for name in _gpu_models(bbm):
        g = ou.golden_model(name)
        for si in range(len(META["models"][name]["sets"])):
            params = g[f"params{si}"]
            m = bbm.BsdfModel(name)
            m.set_parameter_values(params)
            got, flag = _gpu_sample(m, INP["sout"], INP["sxi"])
            _save(f"sample_{name}_{si}", np.concatenate([got, flag[None].astype(np.float32)], 0))
            stats[f"{name}[{si}]"] = _check_samples(bbm, name, params, INP["sout"], INP["sxi"], got, flag,
                                                    g[f"sample{si}"], g[f"sflag{si}"], f"{name}[{si}]")
    _report("sample", stats)


def test_sample_large_batch_vs_reference(bbm):
    n = 1 << 20
    out = bbm.fill_directions(0xBB5EED, 2, 0, n, mode=1)
    xi = torch.rand((2, n), generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
    hout, hxi = out.cpu().numpy(), xi.cpu().numpy()
    stats = {}
    for name in _gpu_models(bbm):
        if name not in ou.oracle_models():
            continue
        m = bbm.BsdfModel(name)
        params = m.parameter_values()
        s = m.sample(out, xi)
        torch.cuda.synchronize()
        got = np.concatenate([s.direction.cpu().numpy(), s.pdf.cpu().numpy()[None]], 0)
        ref, flag = ou.oracle_sample(name, params, hout, hxi, nthreads=8)
        stats[name] = _check_samples(bbm, name, params, hout, hxi, got, s.flag.cpu().numpy(), ref, flag, name)
    _report("sample_large", stats)


EXACT_SAMPLERS = ("CookTorrance", "CookTorranceWalter", "CookTorranceHeitz", "NganCookTorrance", "GGX", "GGXHeitz")


@pytest.mark.parametrize("name", EXACT_SAMPLERS)
def test_exact_mode_sampling(bbm, name):
    """Exact mode's sampler twin (math.hpp exact_sample_t): Beckmann's visible-normal sampler starts its Newton
    steps from glibc's erff / logf, GGX's takes glibc's sinf / cosf of the azimuth (the default: the device
    library's).  Both modes meet the bar or the proofs on the 1M-sample batch, and the twin's directions are within
    1e-6 of the reference on at least as many lanes (checkBsdf's statistics: tests/test_gpu_check.py)."""
    n = 1 << 20
    out = bbm.fill_directions(0xBB5EED, 2, 0, n, mode=1)
    xi = torch.rand((2, n), generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
    hout, hxi = out.cpu().numpy(), xi.cpu().numpy()
    m = bbm.BsdfModel(name)
    params = m.parameter_values()
    ref, rflag = ou.oracle_sample(name, params, hout, hxi, nthreads=8)
    stats = {}
    try:
        for mode in (True, False):
            bbm.set_exact_subnormals(mode)
            s = m.sample(out, xi)
            torch.cuda.synchronize()
            got = np.concatenate([s.direction.cpu().numpy(), s.pdf.cpu().numpy()[None]], 0)
            stats["exact" if mode else "default"] = _check_samples(bbm, name, params, hout, hxi, got,
                                                                   s.flag.cpu().numpy(), ref, rflag, f"{name} {mode}")
    finally:
        bbm.set_exact_subnormals(False)
    ex, de = stats["exact"], stats["default"]
    assert ex["frac_dir_within_1e-6"] >= de["frac_dir_within_1e-6"], stats
    assert ex["dir_lanes_outside_bar"] <= de["dir_lanes_outside_bar"], stats
    _report(f"exact_sample_{name}", stats)


def test_cpp_adapter_drop_in(bbm):
    """backbone/hip C++ adapter: the same bbm::bsdfmodel<> instances (reference template API) on the
    CPU (native backbone) and through bbm::hip::{eval_pdf, sample} on the GPU (tests/cpp)."""
    import subprocess
    exe = os.path.join(ou.ROOT, "tests", "cpp", "_build", "adapter_check")
    if not os.path.exists(exe):
        pytest.skip("tests/cpp/_build/adapter_check not built (needs the reference headers at build time)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    os.makedirs(os.path.join(ou.ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ou.ROOT, "gpurun_out", "adapter_check.jsonl"), "w") as f:
        f.write(r.stdout)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_epd_g1_table_matches_reference(bbm):
    """The EPD shadowing table libbbm_hip builds on the GPU (restating precompute/HolzschuchPacanowski/G1.cpp with
    the FMA contractions of the build that produced the shipped table) against the reference's own
    include/precomputed/holzschuchpacanowski/G1.h: every entry identical (round 5, each op rounded on its own:
    96.4 %; tests/test_oracle.py::test_epd_g1_generator_recipe pins the recipe on the CPU)."""
    import ctypes
    lib = bbm._lib.load()
    n = lib.bbm_hip_epd_g1_table(None, 0)
    assert n == 100 * 1000
    got = np.zeros(n, np.float32)
    assert lib.bbm_hip_epd_g1_table(got.ctypes.data_as(ctypes.c_void_p), n) == n
    ref = ou.ref()
    want = np.zeros(n, np.float32)
    assert ref.bbmref_epd_g1(want.ctypes.data_as(ctypes.c_void_p), n) == n
    exact = float(np.mean(got == want))
    print(f"EPD G1 table: {exact:.5f} of entries identical")
    _report("epd_g1_table", {"entries": n, "frac_identical": exact,
                             "differing": [int(i) for i in np.nonzero(got != want)[0][:16]]})
    assert exact == 1.0


def test_headline_size_parity(bbm):
    """Config 2 at its own size: CookTorrance eval+pdf over the bench's 100 M device-generated pairs (bench.py: seed
    0xBB5EED, upper hemisphere, the default parameters) plus 3 so the scalar tail runs as well, in one launch; a strided
    subset of 2^20 lanes plus the last two quads and the tail copied back and held to the per-lane bar against the
    reference (oracle/_ref).  Both modes, chosen per call (BBM_HIP_CALL_DEFAULT / BBM_HIP_CALL_EXACT) while the
    process-wide switch says the opposite: the exact mode must be bit-identical on the subset."""
    n = 100_000_003
    din = bbm.fill_directions(0xBB5EED, 0, 0, n, mode=0)
    dout = bbm.fill_directions(0xBB5EED, 1, 0, n, mode=0)
    stride = n // (1 << 20)
    idx = np.unique(np.concatenate([np.arange(0, n, stride), np.arange(n - 11, n)]))
    tidx = torch.from_numpy(idx).cuda()
    hin, hout = din[:, tidx].cpu().numpy(), dout[:, tidx].cpu().numpy()
    m = bbm.BsdfModel("CookTorrance")
    params = m.parameter_values()
    ref = ou.oracle_eval_pdf("CookTorrance", params, hin, hout, nthreads=8)
    stats = {}
    prev = bbm.set_exact_subnormals(True)
    try:
        for exact in (True, False):
            bbm.set_exact_subnormals(not exact)       # the per-call bit must win over the process-wide switch
            rgb, pdf = m.eval_pdf(din, dout, exact=exact)
            got = torch.cat([rgb[:, tidx], pdf[tidx][None]]).cpu().numpy()
            del rgb, pdf
            s = check_lanes(got, ref, f"CookTorrance 100M {'exact' if exact else 'default'}",
                            _evalpdf_provers(bbm, "CookTorrance", params, hin, hout, got))
            s["pairs_in_launch"], s["subset_lanes"] = n, int(idx.size)
            if exact:
                assert s["frac_bit_exact"] == 1.0, s
            else:
                # default mode: quotients of subnormal intermediates rounded on the normal grid (values < 1e-30;
                # 99.61 % bit-identical on the 1 M-pair batches at roughness 0.1)
                assert s["frac_bit_exact"] >= 0.99, s
            stats["exact" if exact else "default"] = s
    finally:
        bbm.set_exact_subnormals(prev)
    _report("headline_100m", stats)


def test_bagher_out_of_range_parameters(bbm):
    """Bagher's NDF with parameters outside the attributes' ranges (the reference accepts any alpha / p,
    ndf/sgd.h:56-58): alpha <= 0, alpha = NaN, a negative base with an integer or fractional power, p = 0 -- D takes
    glibc's powf with its negative-base rules, IEEE quotients and the overflowing expf (spectral.hpp), so eval equals
    the reference's floats (NaN for NaN) on every lane, like the in-range parameters."""
    n = 1 << 16
    din = bbm.fill_directions(7, 0, 0, n, mode=0).cpu().numpy()
    dout = bbm.fill_directions(7, 1, 0, n, mode=0).cpu().numpy()
    m = bbm.BsdfModel("Bagher")
    base = m.parameter_values()
    layout = dict((k, i) for i, k in enumerate(["albedo", "K", "Lambda", "c", "theta0", "k", "alpha", "p", "F0", "F1"]))
    cases = {"alpha_neg_int_p": ([-1.0, -0.5, -2.0], [2.0, 3.0, 1.0]),
             "alpha_neg_frac_p": ([-1.0, -0.3, -0.7], [1.5, 0.5, 2.5]),
             "alpha_zero": ([0.0, -0.0, 0.0], [2.0, 1.0, 0.5]),
             "alpha_nan": ([float("nan"), 0.2, float("nan")], [1.0, 1.0, 1.0]),
             "p_zero": ([0.2, 0.3, 0.4], [0.0, 0.0, 0.0])}
    stats = {}
    for tag, (alpha, p) in cases.items():
        params = base.copy()
        params[3 * layout["alpha"]:3 * layout["alpha"] + 3] = alpha
        params[3 * layout["p"]:3 * layout["p"] + 3] = p
        m.set_parameter_values(params)
        got = m.eval(_dev(din), _dev(dout)).cpu().numpy()
        ref = ou.oracle_eval_pdf("Bagher", params, din, dout, nthreads=8)[:3]
        same = (got == ref) | (np.isnan(got) & np.isnan(ref))
        ok = ou.parity_ok(got, ref) | same
        stats[tag] = {"frac_identical": float(same.mean()), "lanes_outside_bar": int((~ok.all(0)).sum())}
        assert ok.all(), f"Bagher {tag}: {stats[tag]}"
    _report("bagher_out_of_range", stats)


def test_he_sampler_backscatter_bit_identical(bbm):
    """The He family's data-driven sampler (ndf/sampler.h:143-181) tabulates hsum(eval(d, d)) at 90 backscatter
    directions; the GPU's evaluations there are the reference's floats on every direction, channel and golden
    parameter set, so the 90-bin CDF -- a serial float prefix sum of them -- is the reference's bit for bit (round 6:
    shadowing S, geometry G, sigma, D, the float complex Fresnel and 1 / (pi z z) each pinned at these directions by
    a diagnostics build, tools/dbg_he_parts.py)."""
    d = ou.sampler_backscatter_dirs().astype(np.float32)
    stats = {}
    for name in ("He", "HeWestin", "HeHolzschuch", "NganHe"):
        g = ou.golden_model(name)
        for si in range(len(META["models"][name]["sets"])):
            params = g[f"params{si}"]
            m = bbm.BsdfModel(name)
            m.set_parameter_values(params)
            got = _gpu_evalpdf(m, d, d)[:3]
            ref = ou.oracle_eval_pdf(name, params, d, d, nthreads=4)[:3]
            same = (got.view(np.uint32) == ref.view(np.uint32))
            stats[f"{name}[{si}]"] = {"directions": int(d.shape[1]), "identical": float(same.mean()),
                                      "differing": [int(i) for i in np.nonzero(~same.all(0))[0][:12]]}
    _report("he_backscatter", stats)
    bad = {k: v for k, v in stats.items() if v["identical"] < 1.0}
    assert not bad, bad
