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
