"""BBM_BACKBONE=hip: the backbone plug-in (backbone/hip/backbone.cmake, backbone/hip/include/backbone.h) and the
host adapter's dispatch (backbone/hip/include/bbm_hip/batch.h), CPU only.

tests/cpp/backbone_check.cpp is compiled against the reference's headers with the HIP backbone first on the
include path, exactly as backbone.cmake sets it up (build() does it here; the binary travels to the GPU box).
It validates floatRGB and doubleRGB with the reference's own BBM_CHECK_CONFIG (bbm/config.h:31-40 ->
BBM_VALIDATE_BACKBONE, core/backbone.h:34-49), instantiates every exported model on both configurations, and
resolves every floatRGB model by type, by string and through a bsdf_ptr to the same libbbm_hip entry and the
reference's own parameter values.  No kernel runs: the GPU side is tests/cpp/adapter_check.cpp
(tests/test_gpu_parity.py::test_cpp_adapter_drop_in).
"""
import json
import os
import re
import subprocess

import pytest

from tests import oracle_util as ou

EXE = os.path.join(ou.ROOT, "tests", "cpp", "_build", "backbone_check")
EXPORTED = 35      # BBM_EXPORT_BSDFMODEL in include/bsdfmodel/*.h and staticmodel/merl.h


@pytest.fixture(scope="module")
def lines():
    if not os.path.exists(EXE):
        pytest.skip("tests/cpp/_build/backbone_check not built (needs the reference headers at build time)")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


def test_every_exported_model_instantiates_on_both_configs(lines):
    head = lines[0]
    assert head["instantiated"] == 2 * (EXPORTED - 1) and head["configs"] == ["floatRGB", "doubleRGB"]
    assert head["checksum_finite"]


def test_dispatch_by_type_string_and_bsdf_ptr(lines):
    models = [x for x in lines if "model" in x]
    assert all(x["ok"] for x in models), [x for x in models if not x["ok"]]
    kernels = {x["kernel"] for x in models if x["entries"] == 1}
    from bbm_amd.models import ATTRIBUTES
    assert set(ATTRIBUTES) <= kernels          # all 34 analytic models resolve to their own kernel
    assert "Aggregate<Lambertian,NganHe>" in kernels
    assert any(x["entries"] == 4 for x in models)    # composed aggregate of four children
    assert lines[-1] == {"failures": 0}


def test_backbone_files_present():
    root = os.path.join(ou.ROOT, "backbone", "hip")
    with open(os.path.join(root, "backbone.cmake")) as f:
        cm = f.read()
    assert re.search(r'set\(BBM_BACKBONE_CONFIGURATIONS "floatRGB" "doubleRGB"\)', cm)
    assert "backbone/hip/include" in cm and "target_link_libraries" in cm
    with open(os.path.join(root, "include", "backbone.h")) as f:
        h = f.read()
    assert "struct floatRGB" in h and "struct doubleRGB" in h and "BBM_BACKBONE_HIP" in h
