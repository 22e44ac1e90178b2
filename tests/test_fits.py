"""Every material of every published fit file (fits/*.fit) through the host mirror's fromString: the same
model kernel and the bit-identical parameter vector the reference's own bbm::fromString gives (fixture
tests/golden/fits.json, written by oracle/gen_fits_golden.py from the reference), and the same rejections
(bagher_sgd.fit holds ten materials with a value beyond the float range, which the reference refuses)."""
import json
import os

import numpy as np
import pytest

from tests import oracle_util as ou

FITS = json.load(open(os.path.join(ou.GOLDEN, "fits.json")))


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    return bbm_amd


@pytest.mark.parametrize("fname", sorted(FITS))
def test_every_fit_line_parses_like_the_reference(bbm, fname):
    for material, s, key, params in FITS[fname]:
        if params is None:
            with pytest.raises(ValueError):
                bbm.fromString(s)
            continue
        m = bbm.fromString(s)
        assert m.name == key, (fname, material, m.name)
        # every published fit is Aggregate(Lambertian, X): each has a fused kernel of its own
        assert isinstance(m, bbm.BsdfModel), (fname, material)
        got = m.parameter_values()
        want = np.asarray(params, np.float32)
        assert got.shape == want.shape and np.array_equal(got, want), (fname, material, got, want)


def test_fits_cover_every_published_file_and_model():
    assert len(FITS) == 14 and sum(len(v) for v in FITS.values()) == 1302
    keys = {row[2] for rows in FITS.values() for row in rows}
    assert "Aggregate<Lambertian,NganHe>" in keys and "Aggregate<Lambertian,Bagher>" in keys


def test_generic_aggregates_parse(bbm):
    m = bbm.fromString("Aggregate(Lambertian(albedo = [0.1, 0.2, 0.3]), CookTorrance(roughness = 0.2), "
                       "GGX(eta = 1.5))")
    assert isinstance(m, bbm.AggregateModel) and m.name == "Aggregate<Lambertian,CookTorrance,GGX>"
    assert m.parameter_values().size == 3 + 5 + 5
    assert str(bbm.fromString(str(m))) == str(m)
    with pytest.raises(ValueError):
        bbm.AggregateModel(bbm.Lambertian())


def test_c_abi_parser_matches_reference_on_every_fit_line():
    """bbm_hip_parse_model (the C-ABI restatement of the reference's runtime fromString, for FFI callers and the
    C++ adapter's bsdf_ptr path) gives the reference's parameter vectors for every fits/*.fit material."""
    import ctypes
    from bbm_amd import _lib
    lib = _lib.load()
    ids = (ctypes.c_int * 8)()
    nps = (ctypes.c_int * 8)()
    buf = (ctypes.c_float * 256)()
    for fname, rows in FITS.items():
        for material, s, key, params in rows:
            k = lib.bbm_hip_parse_model(s.encode(), ids, buf, nps, 8, 256)
            if params is None:
                assert k == _lib.ERR_INVALID_ARG and b"float range" in lib.bbm_hip_last_error(), (fname, material)
                continue
            assert k == 1 and lib.bbm_hip_model_name(ids[0]).decode() == key, (fname, material)
            # every fit is Aggregate(Lambertian, X): the runtime aggregatebsdf of bsdf_import (bsdf_string_convert.h:59)
            assert ids[0] & 0x40000000, (fname, material)
            assert np.array_equal(np.array(buf[:nps[0]], np.float32), np.asarray(params, np.float32)), (fname, material)


def test_c_abi_layouts_equal_python_mirror():
    import ctypes
    from bbm_amd import _lib
    from bbm_amd.models import ATTRIBUTES, attr_size
    lib = _lib.load()
    for name, layout in ATTRIBUTES.items():
        i = lib.bbm_hip_model_id(name.encode())
        want = ",".join(f"{a}:{attr_size(s)}" for a, s in layout)
        assert lib.bbm_hip_model_layout(i).decode() == want, name
    ids = (ctypes.c_int * 8)()
    nps = (ctypes.c_int * 8)()
    buf = (ctypes.c_float * 256)()
    # composed aggregate: one entry per child; positional attributes; defaults for the rest; errors
    k = lib.bbm_hip_parse_model(b"Aggregate(Lambertian([0.1, 0.2, 0.3]), CookTorrance(roughness = 0.2), GGX)",
                                ids, buf, nps, 8, 256)
    assert k == 3 and [lib.bbm_hip_model_name(ids[j]).decode() for j in range(3)] == ["Lambertian", "CookTorrance", "GGX"]
    assert list(nps[:3]) == [3, 5, 5]
    np.testing.assert_array_equal(np.array(buf[:13], np.float32),
                                  np.float32([0.1, 0.2, 0.3, 0.5, 0.5, 0.5, 0.2, 1.3, 0.5, 0.5, 0.5, 0.1, 1.3]))
    assert lib.bbm_hip_parse_model(b"NoSuchModel(a = 1)", ids, buf, nps, 8, 256) == _lib.ERR_INVALID_MODEL
    assert lib.bbm_hip_parse_model(b"CookTorrance(sharpness = 3)", ids, buf, nps, 8, 256) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_parse_model(b"CookTorrance(albedo = [1, 2])", ids, buf, nps, 8, 256) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_parse_model(b"CookTorrance(eta = 1.5", ids, buf, nps, 8, 256) == _lib.ERR_INVALID_ARG
