"""The oracle is pinned before it is trusted (CPU only).

* The C restatement (oracle/port) must reproduce the reference's floatRGB outputs stored in
  tests/golden (generated from the compiled reference headers) bit for bit.
* The reference shim itself (oracle/_ref, if prebuilt) must reproduce the fixtures it wrote.
* Known-answer values printed in the reference's docs (docs/source/use_bsdf.rst:24-43,236-250)
  and the survey's spot value are checked directly.
"""
import numpy as np
import pytest

from tests import oracle_util as ou

META = ou.golden_meta()
INP = ou.golden_inputs()
PORT_MODELS = ou.port_models()


def _sets(name):
    return range(len(META["models"][name]["sets"]))


@pytest.mark.parametrize("name", PORT_MODELS)
def test_port_bit_exact_vs_reference_golden(name):
    g = ou.golden_model(name)
    for si in _sets(name):
        got = ou.port_eval_pdf(name, g[f"params{si}"], INP["pin"], INP["pout"])
        d = ou.ulp_diff(got, g[f"evalpdf{si}"])
        assert d.max() == 0, f"{name} set {si}: {np.count_nonzero(d)} values differ (max {d.max()} ulp)"


@pytest.mark.parametrize("name", PORT_MODELS)
@pytest.mark.parametrize("tag,comp,unit", [("diffuse", 1, 0), ("specular", 2, 0), ("importance", 3, 1)])
def test_port_component_and_unit_masks(name, tag, comp, unit):
    g = ou.golden_model(name)
    got = ou.port_eval_pdf(name, g["params0"], INP["pin"], INP["pout"], component=comp, unit=unit)
    assert ou.ulp_diff(got, g[f"evalpdf_{tag}"]).max() == 0


def test_port_lambertian_sample_bit_exact():
    g = ou.golden_model("Lambertian")
    for si in _sets("Lambertian"):
        got, flag = ou.port_sample("Lambertian", g[f"params{si}"], INP["sout"], INP["sxi"])
        assert ou.ulp_diff(got, g[f"sample{si}"]).max() == 0
        assert np.array_equal(flag.astype(np.uint8), g[f"sflag{si}"])


def test_golden_float_vs_double_spread_is_within_budget():
    """floatRGB vs doubleRGB of the reference itself: the scale of the 1e-5 parity budget."""
    for name in ("CookTorrance", "GGX"):
        g = ou.golden_model(name)
        f, d = g["evalpdf0"].astype(np.float64), g["evalpdf_double"]
        sel = np.abs(d) > 1e-6
        assert (np.abs(f - d)[sel] / np.abs(d[sel])).max() < 1e-5


def test_docs_known_answers_lambertian():
    """docs/source/use_bsdf.rst:24-43 (default Lambertian at in = out = z) and :236-250."""
    z = np.array([[0.0], [0.0], [1.0]], np.float32)
    r = ou.port_eval_pdf("Lambertian", [0.5, 0.5, 0.5], z, z)
    np.testing.assert_allclose(r[:3, 0], [0.159155] * 3, rtol=2e-6)
    np.testing.assert_allclose(r[3, 0], 0.31831, rtol=2e-5)
    r = ou.port_eval_pdf("Lambertian", [0.1, 0.2, 0.3], z, z)
    np.testing.assert_allclose(r[:3, 0], [0.03183099, 0.06366198, 0.09549297], rtol=1e-6)
    got, flag = ou.port_sample("Lambertian", [0.5, 0.5, 0.5], z, np.array([[0.3], [0.7]], np.float32))
    np.testing.assert_allclose(got[:3, 0], [-0.169256, 0.520915, 0.83666], atol=2e-6)
    np.testing.assert_allclose(got[3, 0], 0.266317, rtol=2e-6)
    assert flag[0] == 1


def test_survey_spot_value_cooktorrance():
    """CookTorrance defaults at in = normalize(0.3,0.1,0.9), out = normalize(-0.2,0.05,0.8)
    (normalised in float, as bbm::normalize does)."""
    def nf(v):
        v = np.asarray(v, np.float32)
        s = np.float32(0) + v[0] * v[0]
        s = s + v[1] * v[1]
        s = s + v[2] * v[2]
        return (v * (np.float32(1) / np.sqrt(s, dtype=np.float32))).reshape(3, 1)
    r = ou.port_eval_pdf("CookTorrance", [0.5, 0.5, 0.5, 0.1, 1.3], nf([0.3, 0.1, 0.9]), nf([-0.2, 0.05, 0.8]))
    assert np.float32(r[0, 0]) == np.float32(0.124202915)
    assert np.float32(r[3, 0]) == np.float32(10.7763062)


@pytest.mark.skipif(ou.ref() is None, reason="oracle/_ref not built")
def test_reference_shim_reproduces_its_fixtures():
    for name in META["models"]:
        g = ou.golden_model(name)
        got = ou.ref_eval_pdf(name, g["params0"], INP["pin"], INP["pout"])
        assert ou.ulp_diff(got, g["evalpdf0"]).max() == 0, name


def test_dirgen_counter_property():
    """Slices of one global batch regenerate identically from (seed, offset)."""
    full = ou.dirgen_numpy(7, 0, 0, 1000, mode=1)
    part = ou.dirgen_numpy(7, 0, 600, 400, mode=1)
    assert np.array_equal(full[:, 600:], part)
    n = np.linalg.norm(full.astype(np.float64), axis=0)
    np.testing.assert_allclose(n, 1.0, atol=1e-6)


@pytest.mark.skipif(ou.ref() is None, reason="oracle/_ref not built")
def test_sampler_pdf_restatement_matches_reference():
    """The numpy restatement of the tabulated samplers' pdf (used by the sampler-CDF proof) reproduces the
    reference's own pdf from the reference's own backscatter evaluations (within 1e-5; ~99 % bit-exact)."""
    hb = ou.sampler_backscatter_dirs()
    for name in sorted({'He', 'HeWestin', 'HeHolzschuch', 'NganHe'}):
        g = ou.golden_model(name)
        for si in range(len(ou.golden_meta()["models"][name]["sets"])):
            p = g[f"params{si}"].copy()
            if name == "NganHe":
                p[:3] = 1.0
            bs = ou.oracle_eval_pdf(name, p, hb, hb, nthreads=8)
            want = ou.sampler_pdf(ou.sampler_cdf(bs[:3]), ou.golden_inputs()["pin"], ou.golden_inputs()["pout"])
            assert ou.parity_ok(want, g[f"evalpdf{si}"][3]).all(), f"{name}[{si}]"


def test_config1_lambertian_native_cpu_1m_pairs():
    """BASELINE.json configs[0]: Lambertian eval on the native CPU backbone over 1M (in, out) pairs -- the
    plumbing case without a GPU.  The reference itself (oracle/_ref, native floatRGB) and the C restatement
    agree bit for bit, and both equal albedo / pi on the upper hemisphere (lambertian.h:45-59)."""
    import time
    rng = np.random.default_rng(20240601)
    n = 1_000_000

    def dirs(sphere):
        z = (2 * rng.random(n) - 1 if sphere else rng.random(n)).astype(np.float32)
        ph = (2 * np.pi * rng.random(n)).astype(np.float32)
        s = np.sqrt(np.maximum(1 - z * z, 0)).astype(np.float32)
        return np.ascontiguousarray(np.stack([s * np.cos(ph), s * np.sin(ph), z]).astype(np.float32))

    din, dout = dirs(True), dirs(True)
    albedo = np.float32([0.5, 0.25, 0.125])
    t0 = time.perf_counter()
    got = ou.oracle_eval_pdf("Lambertian", albedo, din, dout, nthreads=4)
    el = time.perf_counter() - t0
    port = ou.port_eval_pdf("Lambertian", albedo, din, dout, nthreads=4)
    np.testing.assert_array_equal(got, port)
    up = (din[2] > 0) & (dout[2] > 0)
    want = np.where(up, (albedo[:, None] / np.float32(np.pi)).astype(np.float32), np.float32(0))
    np.testing.assert_array_equal(got[:3], want)
    assert el < 60, el


def test_expf_restatement_matches_host_libm():
    """bbm_amd/csrc/math.hpp expf_glibc restates glibc's expf (the reference's bbm::exp(float) on x86-64);
    oracle/expf_glibc_check runs the same double steps in C against this host's libm on every 61st float of
    [-110, 90] (the full sweep, stride 1, is 2.24e9 floats and 0 mismatches -- DESIGN.md §4.2)."""
    import os
    import subprocess
    exe = os.path.join(ou.ROOT, "oracle", "_port", "expf_glibc_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ou.ROOT, "oracle"), "expf"], check=True, capture_output=True)
    r = subprocess.run([exe, "61"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert " 0 mismatches" in r.stdout


def _run_check(name, *args):
    import os
    import subprocess
    exe = os.path.join(ou.ROOT, "oracle", "_port", name)
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ou.ROOT, "oracle"), "expf"], check=True, capture_output=True)
    r = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    return r.stdout


def test_powf_logf_restatements_match_host_libm():
    """math.hpp powf_glibc / logf_glibc restate glibc's powf / logf (the reference's bbm::pow / bbm::log of floats);
    oracle/glibcf_check runs the same double steps in C against this host's libm: logf on every positive float, powf
    on 5 x 4e6 random pairs here (the full run, 1e9 pairs, 0 mismatches -- DESIGN.md §4.2).  It also counts how often
    glibc's powf is not the correctly rounded float -- the reason the restatement must be glibc's, not the nearest."""
    out = _run_check("glibcf_check", 4000000)
    assert "logf: 2139095039 positive floats, 0 mismatches" in out, out
    assert "powf: 20000000 (x, y) pairs, 0 mismatches" in out, out


def test_erff_erfcf_restatements_match_host_libm():
    """math.hpp erff_glibc / erfcf_glibc restate glibc's float erf / erfc (fdlibm's s_erff.c); oracle/erfcf_glibc_check
    compares the C restatement with this host's libm on every 31st float bit pattern here (stride 1: all 2^32, 0
    mismatches)."""
    out = _run_check("erfcf_glibc_check", 31)
    assert "erfcf 0 mismatches, erff 0 mismatches" in out, out


def test_sinf_cosf_restatements_match_host_libm():
    """math.hpp sincosf_glibc restates glibc's sinf / cosf (the reference's bbm::cossin of a float, on every sampler
    angle); oracle/sincosf_glibc_check runs the same double steps in C against this host's libm on every 7th float
    with |x| < 120 here (stride 1: all 2.2e9, 0 mismatches)."""
    out = _run_check("sincosf_glibc_check", 7)
    assert "cosf mismatches 0, sinf mismatches 0" in out, out


def test_atan2f_restatement_matches_host_libm():
    """math.hpp atan2f_glibc restates glibc's atan2f (fdlibm's float e_atan2f.c / s_atanf.c; the reference's
    spherical::phi); oracle/atan2f_glibc_check runs the same float steps in C against this host's libm on 3 x 2e6
    random pairs here (3 x 2e7 in DESIGN.md) and every zero / infinity / NaN combination."""
    out = _run_check("atan2f_glibc_check", 2000000)
    assert "0 mismatches" in out, out


def test_theta_restatement_matches_glibc():
    """spectral.hpp theta_of (spherical::theta: float(2 asin(|v - pole| / 2)) in double) by a degree-11 polynomial asin
    with a midpoint guard; oracle/theta_check runs the same double steps against this host's glibc asin for every
    13th float chord length in [0, 2], both hemispheres (stride 1: all 1.07e9, 0 mismatches)."""
    out = _run_check("theta_check", 13)
    assert " 0 mismatches" in out, out


@pytest.mark.skipif(ou.ref() is None, reason="oracle/_ref not built")
def test_epd_g1_generator_recipe():
    """The shipped EPD shadowing table (include/precomputed/holzschuchpacanowski/G1.h, read through the compiled
    reference) is what precompute/HolzschuchPacanowski/G1.cpp prints when GCC contracts its three multiply-adds
    into FMAs (built with FMA available and gnu++20's default -ffp-contract=fast: the whole generated header then
    equals G1.h byte for byte in every entry, found by compiling G1.cpp here under candidate recipes).  The C
    restatement (oracle/port, bbmport_epd_g1_row) with those contractions reproduces sampled rows exactly; without
    them a fifth of a row differs in the 6th printed digit.  libbbm_hip's on-device generator follows the
    contracted recipe (bbm_amd/csrc/inst_epd.hip; GPU: test_epd_g1_table_matches_reference)."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    port, ref = ou.port(), ou.ref()
    want = np.zeros(100000, np.float32)
    assert ref.bbmref_epd_g1(want.ctypes.data_as(ctypes.c_void_p), want.size) == want.size

    def row(args):
        r, contract = args
        out = np.zeros(1000, np.float32)
        assert port.bbmport_epd_g1_row(r, contract, out.ctypes.data_as(ctypes.c_void_p)) == 0
        return np.mean(out == want[r * 1000:(r + 1) * 1000])

    cases = [(0, 1), (2, 1), (17, 1), (54, 1), (99, 1), (2, 0)]
    with ThreadPoolExecutor(6) as ex:
        same = list(ex.map(row, cases))
    assert same[:5] == [1.0] * 5, same
    assert same[5] < 0.9, same
