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
    out = _run(f"bsdfmodel={MODEL}", "test=pdf", "samples=100000", "checkBelowHorizon")
    res = check.test_pdf(bbm.fromString(MODEL), samples=100000, checkBelowHorizon=True, verbose=False)
    v = _nums([l for l in out.splitlines() if l.startswith("PDF has")][0])
    assert v[:4] == [res["negative"][0], res["negative"][1], res["below_horizon"][0], res["below_horizon"][1]]
    _same(v[4], res["mismatch"][0])
    _same(v[5], res["mismatch"][1])


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
