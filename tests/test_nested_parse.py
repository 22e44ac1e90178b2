"""Nested aggregate strings on the CPU (no kernel runs): the C-ABI parser (bbm_hip_parse_model_tree,
bbm_hip_parse_model) and bbm_amd.fromString against the reference's own fromString of the nested aggregate types
(aggregatemodel_base takes any bsdfmodel child, include/bsdfmodel/aggregatemodel.h:22; fromString :192-213)."""
import ctypes

import numpy as np
import pytest

from tests import oracle_util as ou

NESTED = ["Aggregate<Aggregate<Lambertian,Ward>,GGX>", "Aggregate<Aggregate<Lambertian,CookTorrance>,Ward>",
          "Aggregate<GGX,Aggregate<Phong,Aggregate<Ward,OrenNayar>>>"]


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    return bbm_amd


def _tree(lib, s):
    ids = (ctypes.c_int * 64)()
    nk = (ctypes.c_int * 64)()
    npar = (ctypes.c_int * 64)()
    buf = np.zeros(4096, np.float32)
    k = lib.bbm_hip_parse_model_tree(s.encode(), ids, nk, buf.ctypes.data_as(ctypes.c_void_p), npar, 64, buf.size)
    return k, list(ids[:max(k, 0)]), list(nk[:max(k, 0)]), list(npar[:max(k, 0)]), buf


RUNTIME = 0x40000000     # BBM_HIP_RUNTIME_AGGREGATE: a fused aggregate with aggregatebsdf semantics
AGG_BSDF = -101          # BBM_HIP_AGGREGATE_BSDF: a composed runtime aggregate (aggregatebsdf.h)


def _names(lib, ids):
    return ["*" if i == AGG_BSDF else lib.bbm_hip_model_name(i).decode() for i in ids]


needs_ref = pytest.mark.skipif(ou.ref() is None, reason="oracle/_ref not built")


@needs_ref
@pytest.mark.parametrize("key", NESTED)
def test_parse_tree_matches_reference_fromstring(bbm, key):
    lib = bbm._lib.load()
    p = ou.ref_default_params(key)
    p = (p * np.float32(0.875)).astype(np.float32)
    s = ou.ref_to_string(key, p)
    k, ids, nk, npar, buf = _tree(lib, s)
    assert k > 1
    want = ou.ref_from_string(key, s)
    assert np.array_equal(buf[:sum(npar)], want)        # the values the reference reads, leaves in preorder
    assert ids[0] == AGG_BSDF and nk[0] >= 2


def test_parse_tree_structure(bbm):
    lib = bbm._lib.load()
    k, ids, nk, npar, _ = _tree(lib, "Aggregate(Aggregate(Lambertian, Ward), GGX)")
    assert (k, _names(lib, ids), nk, npar) == (5, ["*", "*", "Lambertian", "Ward", "GGX"], [2, 2, 0, 0, 0], [0, 0, 3, 5, 5])
    # a fused inner aggregate stays one registry entry -- the runtime aggregate of a string (bsdf_string_convert.h:59)
    k, ids, nk, npar, _ = _tree(lib, "Aggregate(Aggregate(Lambertian, CookTorrance), Ward)")
    assert (k, _names(lib, ids), nk) == (3, ["*", "Aggregate<Lambertian,CookTorrance>", "Ward"], [2, 0, 0])
    assert ids[1] & RUNTIME and not ids[2] & RUNTIME
    # no composed aggregate: one node
    k, ids, nk, npar, _ = _tree(lib, "Aggregate(Lambertian, CookTorrance)")
    assert (k, _names(lib, ids), nk, npar) == (1, ["Aggregate<Lambertian,CookTorrance>"], [0], [8])
    assert ids[0] & RUNTIME
    # a runtime flag on a single model is not a model
    assert lib.bbm_hip_model_name(lib.bbm_hip_model_id(b"Ward") | RUNTIME) is None


def test_flat_parser_rejects_nested_composed_and_accepts_fused_children(bbm):
    lib = bbm._lib.load()
    ids = (ctypes.c_int * 16)()
    npar = (ctypes.c_int * 16)()
    buf = np.zeros(1024, np.float32)
    ptr = buf.ctypes.data_as(ctypes.c_void_p)
    # a composed aggregate inside another: refused (not flattened), with the tree parser named in the message
    rc = lib.bbm_hip_parse_model(b"Aggregate(Aggregate(Lambertian, Ward), GGX)", ids, ptr, npar, 16, buf.size)
    assert rc == bbm._lib.ERR_UNSUPPORTED and b"parse_model_tree" in lib.bbm_hip_last_error()
    # a fused child is a registry entry like any other
    rc = lib.bbm_hip_parse_model(b"Aggregate(Aggregate(Lambertian, GGX), Ward)", ids, ptr, npar, 16, buf.size)
    assert rc == 2 and _names(lib, ids[:2]) == ["Aggregate<Lambertian,GGX>", "Ward"] and list(npar[:2]) == [8, 5]
    assert ids[0] & RUNTIME


def test_python_fromstring_nested(bbm):
    m = bbm.fromString("Aggregate(Aggregate(Lambertian(albedo = 0.25), Ward(roughness = [0.2, 0.3])), GGX)")
    assert isinstance(m, bbm.AggregateModel) and isinstance(m._children[0], bbm.AggregateModel)
    assert str(m).startswith("Aggregate(Aggregate(Lambertian(albedo = [0.25, 0.25, 0.25]), Ward(")
    assert m.parameter_values().size == 13
    m2 = bbm.fromString(str(m))
    assert np.array_equal(m2.parameter_values(), m.parameter_values())
    f = bbm.fromString("Aggregate(Aggregate(Lambertian, GGX), Ward)")
    assert isinstance(f._children[0], bbm.BsdfModel) and f._children[0].name == "Aggregate<Lambertian,GGX>"
    v = m.parameter_values() * np.float32(0.5)
    m.set_parameter_values(v)
    assert np.array_equal(m.parameter_values(), v)


def test_aggregate_children_are_copies(bbm):
    a = bbm.Lambertian(albedo=0.5)
    agg = bbm.Aggregate(a, bbm.Ward(), fused=False)
    a.set_attribute("albedo", 0.1)
    assert agg.parameter_values()[0] == np.float32(0.5)
    outer = bbm.Aggregate(agg, bbm.GGX())
    agg.set_parameter_values(agg.parameter_values() * 0)
    assert outer.parameter_values()[0] == np.float32(0.5)


@pytest.mark.parametrize("s", [
    "CookTorrance(albedo = [0.6, 0.5, 0.4], roughness = 0.25, eta = 1.6)",
    "Aggregate(Lambertian(albedo = [0.2, 0.3, 0.4]), CookTorrance(roughness = 0.3))",
    "Aggregate(Lambertian(albedo = [0.2, 0.3, 0.4]), CookTorrance(roughness = 0.3), GGX(roughness = 0.15))",
    "Aggregate(Aggregate(Lambertian(albedo = [0.25, 0.25, 0.25]), Ward(roughness = [0.2, 0.3])), "
    "Aggregate(Lambertian(albedo = [0.1, 0.2, 0.1]), GGX(roughness = 0.2)), OrenNayar)",
])
def test_parse_model_matches_fromstring(bbm, s):
    """bbm_amd.parse_model (the C-ABI parser) builds the same models as the Python fromString."""
    def flat(m):
        if isinstance(m, bbm.AggregateModel):
            return ("*", m.runtime, [flat(c) for c in m._children])
        return (m.name, m.model_id, m.runtime, m.parameter_values().tolist())
    assert flat(bbm.parse_model(s)) == flat(bbm.fromString(s))


def test_fit_material_through_the_c_parser(bbm):
    """Config 5's material comes from the fits/ line itself (tools/bench_configs.FIT_LINE, fits/bagher_sgd.fit:3)
    parsed by the library's C parser, and equals the reference's fromString of that line (tests/golden/fits.json)."""
    import json
    import os
    from tools import bench_configs
    name, m = bench_configs.fit_material()
    assert name == "alum-bronze" and m.name == "Aggregate<Lambertian,Bagher>" and m.runtime
    with open(os.path.join(os.path.dirname(__file__), "golden", "fits.json")) as f:
        row = next(r for r in json.load(f)["bagher_sgd.fit"] if r[0] == name)
    assert np.array_equal(m.parameter_values(), bbm.fromString(row[1]).parameter_values())
