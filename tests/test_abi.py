"""The C-ABI boundary and the host-side mirror of the reference interface (CPU only: no kernel runs).

* libbbm_hip.so loads and exports every symbol declared in include/bbm_hip.h;
* the registry (names, parameter counts, defaults, bounds) matches the reference's own values
  recorded in tests/golden/models.json;
* toString / fromString reproduce bbm::toString byte for byte for every model and parameter set;
* argument validation fails loudly with the reference's error categories before any launch.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from tests import oracle_util as ou

ROOT = ou.ROOT
META = ou.golden_meta()


def _header_symbols():
    with open(os.path.join(ROOT, "include", "bbm_hip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(bbm_hip_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    from bbm_amd import _lib
    return _lib.load()


def test_header_symbols_exported(lib):
    syms = _header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/bbm_hip.h but not exported"


def test_binding_covers_header():
    from bbm_amd import _lib
    assert set(_header_symbols()) == set(_lib.SIGNATURES)


def test_abi_version(lib):
    assert lib.bbm_hip_abi_version() == 12


def test_f64_registry(lib):
    """doubleRGB kernels: the microfacet family, the diffuse models and their Aggregate(Lambertian, X) fits."""
    has = {lib.bbm_hip_model_name(i).decode(): lib.bbm_hip_model_has_f64(i) for i in range(lib.bbm_hip_num_models())}
    for name in ("Lambertian", "OrenNayar", "CookTorrance", "GGX", "CookTorranceHeitz", "Ribardiere",
                 "LowMicrofacetFit", "Aggregate<Lambertian,CookTorrance>", "Aggregate<Lambertian,NganCookTorrance>"):
        assert has[name] == 1, name
    for name in ("Ward", "AshikhminShirleyFull", "LowSmooth", "Aggregate<Lambertian,NganWard>", "Bagher",
                 "Aggregate<Lambertian,Bagher>", "EPD", "He", "HeWestin", "HeHolzschuch", "NganHe",
                 "Aggregate<Lambertian,NganHe>"):
        assert has[name] == 1, name
    assert has["Merl"] == 0      # measured data: its table is the floatRGB merl_data's
    assert lib.bbm_hip_model_has_f64(10_000) == -1
    # a model without doubleRGB kernels is refused before anything is launched
    p = (ctypes.c_double * 7)()
    mid = lib.bbm_hip_model_id(b"Merl")
    assert lib.bbm_hip_eval_pdf_f64(mid, p, 2, None, None, None, None, None, None, None, 0, 3, 0,
                                    None, None, None, None, None) == -3


def test_registry_matches_reference(lib):
    from bbm_amd.models import nparams
    names = [lib.bbm_hip_model_name(i).decode() for i in range(lib.bbm_hip_num_models())]
    assert "CookTorrance" in names and "GGX" in names and "Lambertian" in names
    for i, name in enumerate(names):
        if name == "Merl":        # measured data, no attributes in the reference: tests/test_merl.py
            continue
        ref = META["models"][name]
        assert lib.bbm_hip_model_id(name.encode()) == i
        k = lib.bbm_hip_model_nparams(i)
        assert k == ref["nparams"] == nparams(name)
        buf = (ctypes.c_float * k)()
        for which, key in ((0, "defaults"), (1, "lower"), (2, "upper")):
            assert lib.bbm_hip_model_params(i, which, buf, k) == k
            np.testing.assert_array_equal(np.array(buf[:], np.float32), np.array(ref[key], np.float32), err_msg=f"{name} {key}")


def _composed_children(name):
    """Children of a golden aggregate that has no fused registry entry (composed path, bbm_hip_aggregate_*)."""
    from bbm_amd.models import AGGREGATES
    if not name.startswith("Aggregate<") or name in AGGREGATES:
        return None
    return name[len("Aggregate<"):-1].split(",")


def test_python_mirror_layout_covers_every_reference_model():
    from bbm_amd.models import AGGREGATES, ATTRIBUTES, nparams
    for name, ref in META["models"].items():
        kids = _composed_children(name)
        if kids is not None:     # composed aggregate: the children's vectors in order
            assert all(k in ATTRIBUTES for k in kids) and sum(nparams(k) for k in kids) == ref["nparams"], name
            continue
        assert name in ATTRIBUTES or name in AGGREGATES, name
        assert nparams(name) == ref["nparams"], name


def test_param_attrs_match_reference(lib):
    """bsdf_attr flags per parameter == what bbm::parameter_values(model, flag) selects in the reference."""
    names = [lib.bbm_hip_model_name(i).decode() for i in range(lib.bbm_hip_num_models())]
    composed = {n for n in META["models"] if _composed_children(n) is not None}
    assert set(names) - {"Merl"} == set(META["models"]) - composed
    for name in composed:     # an aggregate's flags are its children's, in order
        flags = []
        for kid in _composed_children(name):
            buf = (ctypes.c_uint32 * 64)()
            k = lib.bbm_hip_model_param_attrs(names.index(kid), buf, 64)
            flags += [int(buf[j]) for j in range(k)]
        assert flags == META["models"][name]["attrs"], name
    for i, name in enumerate(names):
        if name == "Merl":        # measured data, no attributes in the reference: tests/test_merl.py
            continue
        ref = META["models"][name]["attrs"]
        buf = (ctypes.c_uint32 * 64)()
        assert lib.bbm_hip_model_param_attrs(i, buf, 64) == len(ref)
        assert [int(buf[j]) for j in range(len(ref))] == ref, name


def test_fit_abi_validation(lib):
    from bbm_amd import _lib, fit
    lin = fit.spherical_linearizer((8, 5), (6, 4))
    assert lin.size() == 8 * 5 * 6 * 4
    assert fit.merl_linearizer().size() == 90 * 90 * 180
    bad = fit.spherical_linearizer((0, 5), (6, 4))
    n = ctypes.c_uint64()
    assert lib.bbm_hip_linearizer_size(ctypes.byref(bad), ctypes.byref(n)) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_loss_workspace_size(36) >= 36 * 8
    agg = lib.bbm_hip_model_id(b"Aggregate<Lambertian,Bagher>")
    assert agg >= 0 and lib.bbm_hip_model_nparams(agg) == 33
    # wrong parameter count, unknown loss, missing workspace: rejected before any launch
    assert lib.bbm_hip_loss(agg, None, 30, 4, ctypes.byref(lin), 0, 16, None, None, None, 3, 3, 0, None, None, 0,
                            None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_loss(agg, None, 33, 4, ctypes.byref(lin), 0, 16, None, None, None, 9, 3, 0, None, None, 0,
                            None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_loss(agg, None, 33, 4, ctypes.byref(lin), 0, lin.size() + 1, None, None, None, 3, 3, 0, None,
                            None, 0, None) == _lib.ERR_INVALID_ARG
    assert b"out of bounds" in lib.bbm_hip_last_error()


def test_aggregate_mirror():
    import bbm_amd
    fitted = bbm_amd.Aggregate(bbm_amd.Lambertian(), bbm_amd.Bagher())
    assert fitted.name == "Aggregate<Lambertian,Bagher>"
    # bsdf_attr::All selects the 18 non-Dependent parameters (compass's P)
    assert len(fitted.parameter_indices()) == 18
    assert [c.name for c in fitted.children()] == ["Lambertian", "Bagher"]
    s = META["models"]["Aggregate<Lambertian,Bagher>"]["strings"][1]
    assert str(bbm_amd.fromString(s)) == s


@pytest.mark.parametrize("name", sorted(META["models"]))
def test_to_string_matches_bbm_toString(name):
    from bbm_amd.models import to_string
    g = ou.golden_model(name)
    for si, s in enumerate(META["models"][name]["strings"]):
        assert to_string(name, g[f"params{si}"]) == s


def test_from_string_round_trip_and_named_args():
    import bbm_amd
    for name in bbm_amd.model_names():
        for s in META["models"].get(name, {"strings": []})["strings"]:
            m = bbm_amd.fromString(s)
            assert str(m) == s
    m = bbm_amd.fromString("CookTorrance(eta = 1.5, roughness = 0.2)")
    np.testing.assert_array_equal(m.parameter_values(), np.float32([0.5, 0.5, 0.5, 0.2, 1.5]))
    m = bbm_amd.CookTorrance(albedo=0.25, eta=2.0)
    assert str(m) == "CookTorrance(albedo = [0.25, 0.25, 0.25], roughness = 0.1, eta = 2)"
    assert m.attribute("eta") == np.float32(2.0)
    with pytest.raises(ValueError):
        bbm_amd.fromString("NoSuchModel(a = 1)")
    with pytest.raises(TypeError):
        bbm_amd.CookTorrance(sharpness=3)


def test_errors_before_launch(lib):
    from bbm_amd import _lib
    p = (ctypes.c_float * 5)(*[0.5, 0.5, 0.5, 0.1, 1.3])
    # unknown model id -> BBM_HIP_ERR_INVALID_MODEL
    assert lib.bbm_hip_eval(99, p, 5, *([None] * 7), 0, 3, 0, None, None, None, None) == _lib.ERR_INVALID_MODEL
    assert b"unknown model" in lib.bbm_hip_last_error()
    # wrong parameter count -> BBM_HIP_ERR_INVALID_ARG
    ct = lib.bbm_hip_model_id(b"CookTorrance")
    assert lib.bbm_hip_eval(ct, p, 4, *([None] * 7), 0, 3, 0, None, None, None, None) == _lib.ERR_INVALID_ARG
    assert b"expected 5 parameters" in lib.bbm_hip_last_error()
    # NULL direction pointers with n > 0 -> BBM_HIP_ERR_INVALID_ARG (nothing launched)
    assert lib.bbm_hip_eval_pdf(ct, p, 5, *([None] * 7), 16, 3, 0, None, None, None, None, None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_model_id(b"Nope") == _lib.ERR_INVALID_MODEL
    # n == 0 is a no-op
    assert lib.bbm_hip_eval_pdf(ct, p, 5, *([None] * 7), 0, 3, 0, None, None, None, None, None) == 0
    with pytest.raises(_lib.BackboneError):
        _lib.check(-1)
