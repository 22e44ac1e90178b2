"""The reference's complex Fresnel (include/bbm/fresnel_complex.h:38-63) rounds differently per instantiation, and
the device restatements follow each (CPU check against the reference itself, through reflectance = F / pi * 4.0 /
norm, he.h:236 and microfacet.h:182-196):

* VALUE = Spectrum (the He family, he.h:116, 490-496): the native backbone's array arithmetic -- a double scalar on
  the left of an array converts to float first (backbone/native/include/backbone/array.h:95) -- so every step is a
  float op (bbm_amd/csrc/he.hpp FresnelComplexRGB);
* VALUE = Value (EPD, holzschuchpacanowski.h:40): `0.5 * float` is a double, so a, Rs and Rp are doubles, rounded
  to float once at the return (bbm_amd/csrc/epd.hpp FresnelComplex).

Both restated in numpy here and compared bit for bit with the reference's reflectance on 20 000 directions per golden
parameter set; the other reading of each (round 4's device code) is shown to differ, so the test pins the choice."""
import numpy as np
import pytest

from tests import oracle_util as ou

pytestmark = pytest.mark.skipif(ou.ref() is None, reason="oracle/_ref not built")
f = np.float32


def _dirs(n=20000):
    z = np.random.default_rng(0).uniform(0.001, 1, n).astype(f)
    return z, np.stack([np.sqrt(1 - z * z).astype(f), np.zeros(n, f), z]).astype(f)


def fresnel_spectrum(n, k, cs):
    """fresnel::complex<CONF, Spectrum>: float array arithmetic throughout"""
    c2 = (cs * cs).astype(f)
    s2 = (f(1) - c2).astype(f)
    n2, k2 = f(n * n), f(k * k)
    temp = ((n2 - k2) - s2).astype(f)
    a2b2 = np.sqrt(np.maximum((temp * temp + (n2 * f(4)) * k2).astype(f), f(0))).astype(f)
    a = np.sqrt(np.maximum(((a2b2 + temp) * f(0.5)).astype(f), f(0))).astype(f)
    a2c = ((a * f(2)) * cs).astype(f)
    rs = (((a2b2 - a2c) + c2) / ((a2b2 + a2c) + c2)).astype(f)
    ca = (c2 * a2b2).astype(f)
    rp = ((rs * (ca - (a2c - s2) * s2)) / (ca + (a2c + s2) * s2)).astype(f)
    return ((rs + rp) * f(0.5)).astype(f)


def fresnel_value(n, k, cs, round_rs=False):
    """fresnel::complex<CONF, Value>: a, Rs, Rp in double, one rounding at the return (round_rs: round 4's reading)"""
    c2 = (cs * cs).astype(f)
    s2 = (f(1) - c2).astype(f)
    n2, k2 = f(n * n), f(k * k)
    temp = ((n2 - k2) - s2).astype(f)
    a2b2 = np.sqrt(np.maximum((temp * temp + (f(4) * n2) * k2).astype(f), f(0))).astype(f)
    a = np.sqrt(np.maximum(0.5 * (a2b2 + temp).astype(f).astype(np.float64), 0))
    a2c = 2 * a * cs.astype(np.float64)
    rs = (a2b2.astype(np.float64) - a2c + c2) / (a2b2.astype(np.float64) + a2c + c2)
    if round_rs:
        rs = rs.astype(f).astype(np.float64)
    ca = (c2 * a2b2).astype(f).astype(np.float64)
    rp = rs * (ca - (a2c - s2) * s2) / (ca + (a2c + s2) * s2)
    if round_rs:
        rp = rp.astype(f).astype(np.float64)
    return (0.5 * (rs + rp)).astype(f)


@pytest.mark.parametrize("name", ["He", "HeWestin", "HeHolzschuch"])
def test_he_fresnel_is_float_array_arithmetic(name):
    z, dout = _dirs()
    g = ou.golden_model(name)
    for si in range(len(ou.golden_meta()["models"][name]["sets"])):
        p = g[f"params{si}"]
        ref = ou.ref_reflectance(name, p, dout)
        n, k = p[2:5], p[5:8]
        got = np.stack([((fresnel_spectrum(n[c], k[c], z) / f(np.pi)).astype(f).astype(np.float64) * 4.0).astype(f)
                        for c in range(3)])
        assert np.array_equal(got, ref), f"{name}[{si}]: {np.mean(got == ref)} bit-identical"


def test_epd_fresnel_keeps_double_quotients():
    z, dout = _dirs()
    g = ou.golden_model("EPD")
    differs = False
    for si in range(len(ou.golden_meta()["models"]["EPD"]["sets"])):
        p = g[f"params{si}"]
        ref = ou.ref_reflectance("EPD", p, dout)[0]
        # Walter normalisation: F / 4.0 * 4.0 in double (microfacet.h:193)
        got = (fresnel_value(p[2], p[3], z).astype(np.float64) / 4.0 * 4.0).astype(f)
        assert np.array_equal(got, ref), f"EPD[{si}]: {np.mean(got == ref)} bit-identical"
        old = (fresnel_value(p[2], p[3], z, round_rs=True).astype(np.float64) / 4.0 * 4.0).astype(f)
        differs |= not np.array_equal(old, ref)
    assert differs
