"""The C++ checkBsdf command line on the HIP backbone (backbone/hip/bin/checkBsdf.cpp, built by tests/cpp/Makefile
into tests/cpp/_build/checkBsdf): the reference's `key=value` CLI (bin/checkBsdf.cpp:420-479) over bbm_hip/check.h.
Its printed statistics equal the Python driver's (bbm_amd.check, the same kernels and draws) to the printed digits,
and its option handling follows the reference (invalid keywords, unknown tests, missing test).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from tests import oracle_util as ou

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

EXE = os.path.join(ou.ROOT, "tests", "cpp", "_build", "checkBsdf")
NUM = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?|nan|inf"


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    if not os.path.exists(EXE):
        pytest.skip("tests/cpp/_build/checkBsdf not built (needs the reference headers at build time)")
    return bbm_amd


def _run(*args):
    r = subprocess.run([EXE, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _nums(line):
    return [float(x) for x in re.findall(NUM, line)]


def _same(got, want):
    # std::cout's default 6 significant digits
    want = float(f"{float(want):.6g}")
    assert got == pytest.approx(want, rel=2e-6, abs=1e-30), (got, want)


MODEL = "Aggregate(Lambertian(albedo=[0.2,0.3,0.4]), CookTorrance(roughness=0.3), GGX(roughness=0.2))"


def test_reflectance_matches_python_driver(bbm):
    from bbm_amd import check
    out = _run(f"bsdfmodel={MODEL}", "test=reflectance", "samples=200000", "theta=3")
    lines = [l for l in out.splitlines() if l.startswith(" out = ")]
    assert len(lines) == 3
    res = check.test_reflectance(bbm.fromString(MODEL), samples=200000, theta=3, verbose=False)
    for t, l in enumerate(lines):
        v = _nums(l)
        for c in range(3):
            _same(v[3 + c], res["estimate"][t][c])
            _same(v[6 + c], res["reflectance"][t][c])


def test_pdf_int_and_pdf_match_python_driver(bbm):
    from bbm_amd import check
    out = _run("bsdfmodel=CookTorrance(roughness=0.25)", "test=pdfInt", "samples=100000", "trials=4", "seed=99")
    lines = [l for l in out.splitlines() if l.startswith(" Integral = ")]
    res = check.test_pdf_int(bbm.fromString("CookTorrance(roughness=0.25)"), samples=100000, trials=4, seed=99,
                             verbose=False)
    assert len(lines) == 4
    for k, l in enumerate(lines):
        v = _nums(l)
        _same(v[0], res["integral"][k][0])
        _same(v[1], res["integral"][k][1])
        for c in range(3):
            _same(v[2 + c], res["directions"][k][c])
    # test=pdf runs the reference's loop (float mismatch sums in sample order, stopping at maxError): with maxError
    # out of reach it sees every sample the GPU statistic sees; its uniform directions come from the reference's
    # host code (the kernel's from the device's), so a count may move by a borderline sample
    out = _run(f"bsdfmodel={MODEL}", "test=pdf", "samples=100000", "checkBelowHorizon", "maxError=1000000")
    res = check.test_pdf(bbm.fromString(MODEL), samples=100000, checkBelowHorizon=True, verbose=False)
    v = _nums([l for l in out.splitlines() if l.startswith("PDF has")][0])
    want = [res["negative"][0], res["negative"][1], res["below_horizon"][0], res["below_horizon"][1]]
    assert v[:2] == want[:2] and all(abs(a - b) <= 2 + 1e-3 * b for a, b in zip(v[2:4], want[2:4])), (v, want)
    for k in range(2):
        assert v[4 + k] == pytest.approx(res["mismatch"][k], rel=1e-3, abs=1e-9)
    # the default maxError = 10 stops the loop at the 10th below-horizon sample, each printed (checkBsdf.cpp:219-233)
    out = _run(f"bsdfmodel={MODEL}", "test=pdf", "samples=100000", "checkBelowHorizon")
    below = [l for l in out.splitlines() if l.startswith(" Sampled direction ") and "below horizon for" in l]
    v = _nums([l for l in out.splitlines() if l.startswith("PDF has")][0])
    assert max(v[2], v[3]) == 10 and len(below) == v[2] + v[3], out


def test_sample_and_symmetry_match_python_driver(bbm):
    from bbm_amd import check
    m = "Ward(roughness=[0.3,0.2])"
    out = _run(f"bsdfmodel={m}", "test=sample", "samples=50000", "pdfSamples=512", "trials=2")
    res = check.test_sample(bbm.fromString(m), pdfSamples=512, samples=50000, trials=2, verbose=False)
    chi = [l for l in out.splitlines() if l.startswith(" Chi2 for ")]
    assert len(chi) == 2
    for k, l in enumerate(chi):
        v = _nums(l[len(" Chi2 for "):])
        _same(v[3], res["trials"][k]["chi2"])
        assert int(v[4]) == res["trials"][k]["df"]
    out = _run(f"bsdfmodel={m}", "test=reciprocity", "samples=100000")
    res = check.test_reciprocity(bbm.fromString(m), samples=100000, verbose=False)
    rad = _nums([l for l in out.splitlines() if l.startswith("Radiance")][0])
    for c in range(3):
        _same(rad[c], res["radiance"]["average"][c])
        _same(rad[3 + c], res["radiance"]["max"][c])


def test_cli_options_follow_reference(bbm):
    out = _run("bsdfmodel=Lambertian", "test=pdfInt", "samples=10", "bogus=1")
    assert "ERROR: invalid keywords:" in out and "bogus" in out
    out = _run("bsdfmodel=Lambertian", "test=nothing")
    assert "Unrecognized test: 'nothing'" in out
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "Usage:" in r.stdout
    r = subprocess.run([EXE, "bsdfmodel=NotAModel", "test=pdf"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "ERROR" in r.stdout


def _cli_oracle(tree, test, opts, seed=5489):
    """The reference's own checkBsdf test loop (oracle/ref_cli.cpp) on the reference's bsdf_ptr: printed text.
    test: 0 reflectance, 1 pdf, 2 reciprocity, 3 adjoint, 4 pdfInt, 5 sample; opts as bbmref_cli_test documents."""
    import ctypes
    lib = ou.ref()
    k, names, nk, params, nps = ou.runtime_tree(tree)
    o = np.zeros(8, np.uint64)
    o[:len(opts)] = opts
    buf = ctypes.create_string_buffer(1 << 20)
    n = lib.bbmref_cli_test(k, names, nk, params.ctypes.data_as(ctypes.c_void_p), nps, test,
                            o.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(seed), buf, len(buf))
    assert 0 <= n < len(buf)
    return buf.value.decode()


def _diff_cli(got, want):
    """Line by line: identical text between the numbers, numbers equal to std::cout's 6 digits (one unit in the last
    printed digit allowed where a per-sample value is not the reference's float).  Returns the count of identical
    lines."""
    g, w = got.strip().splitlines(), want.strip().splitlines()
    assert len(g) == len(w), f"{len(g)} lines vs the reference's {len(w)}:\n{got}\n---\n{want}"
    same = 0
    for a, b in zip(g, w):
        assert re.sub(NUM, "#", a) == re.sub(NUM, "#", b), (a, b)
        na, nb = _nums(a), _nums(b)
        for x, y in zip(na, nb):
            assert x == pytest.approx(y, rel=2e-5, abs=1e-30), (a, b)
        same += a == b
    return same


CT = ("CookTorrance", [0.5, 0.5, 0.5, 0.3, 1.3])
LAMB = ("Lambertian", [0.5, 0.5, 0.5])
WARD = ("Ward", [0.5, 0.5, 0.5, 0.3, 0.2])
CLI_CASES = {
    # grazing uniform directions: microfacet reflection sends some samples below the horizon; maxError = 4 stops the
    # loop at the 4th of one kind, after printing each
    "pdf_ct_below": (["bsdfmodel=CookTorrance(roughness=0.5)", "test=pdf", "samples=20000", "maxError=4",
                      "checkBelowHorizon"], ("CookTorrance", [0.5, 0.5, 0.5, 0.5, 1.3]), 1, [20000, 4, 1, 0]),
    "pdf_lambertian_sphere": (["bsdfmodel=Lambertian", "test=pdf", "samples=30000", "sampleSphere", "checkBelowHorizon"],
                              LAMB, 1, [30000, 10, 1, 1]),
    "refl_lambertian": (["bsdfmodel=Lambertian", "test=reflectance", "samples=40000", "theta=3"], LAMB, 0, [40000, 3, 0]),
    "refl_ct_importance": (["bsdfmodel=CookTorrance(roughness=0.3)", "test=reflectance", "samples=40000", "theta=2",
                            "importanceSampling"], CT, 0, [40000, 2, 1]),
    "reciprocity_ward": (["bsdfmodel=Ward(roughness=[0.3,0.2])", "test=reciprocity", "samples=30000"], WARD, 2, [30000]),
    "adjoint_ct": (["bsdfmodel=CookTorrance(roughness=0.3)", "test=adjoint", "samples=30000"], CT, 3, [30000]),
    "pdfint_ct": (["bsdfmodel=CookTorrance(roughness=0.3)", "test=pdfInt", "samples=20000", "trials=3"], CT, 4,
                  [20000, 3, 0]),
    "sample_ct": (["bsdfmodel=CookTorrance(roughness=0.3)", "test=sample", "pdfSamples=64", "samples=20000", "theta=5",
                   "phi=8", "trials=2"], CT, 5, [64, 20000, 5, 8, 2, 0, 0]),
}


@pytest.mark.parametrize("case", list(CLI_CASES))
def test_cli_mt19937_matches_reference(bbm, case):
    """rng=mt19937: the CLI consumes the reference's std::mt19937 draw sequence and runs the reference's loop order,
    so its printed lines are the reference's (oracle/ref_cli.cpp runs the reference's test on the reference's
    bsdf_ptr with the same seed): the same lines -- the pdf test's per-failure lines and its stop at maxError
    included -- and the same numbers, for every checkBsdf test."""
    seed = 1234
    args, tree, test, opts = CLI_CASES[case]
    got = _run(*args, "rng=mt19937", f"seed={seed}")
    ref = _cli_oracle(tree, test, opts, seed=seed)
    same = _diff_cli(got, ref)
    print(f"{case}: {same} of {len(ref.strip().splitlines())} lines identical\n{got}")
    if case == "pdf_ct_below":
        assert "below horizon for" in ref and ref.count("below horizon for") <= 2 * 4
