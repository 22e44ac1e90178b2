"""The drop-in through the reference's own CMake (CPU only, needs /root/reference and cmake; this container).

A copy of the reference tree gets backbone/hip dropped in (the only change a maintainer makes),
and a consumer project (tests/cmake) adds it with BBM_BACKBONE=hip: the reference's CMakeLists.txt creates the
${BBM_NAME} INTERFACE target (CMakeLists.txt:77), setup_backbone() (cmake/bbm_helpers.cmake:21-41) includes
backbone/hip/backbone.cmake, and the consumer TU compiles against that target and links libbbm_hip.so through it.
The reference tree itself is never written (its configure step generates include/bbm_bsdfmodels.h in the copy)."""
import json
import os
import shutil
import subprocess

import pytest

from tests import oracle_util as ou

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "cmake")) or shutil.which("cmake") is None,
                                reason="needs the reference tree and cmake (build container only)")


def test_backbone_plugs_into_reference_cmake(tmp_path):
    src = tmp_path / "bbm"
    shutil.copytree(REF, src, ignore=shutil.ignore_patterns(".git"))
    shutil.copytree(os.path.join(ou.ROOT, "backbone", "hip"), src / "backbone" / "hip")
    build = tmp_path / "build"
    cfg = subprocess.run(["cmake", "-S", os.path.join(ou.ROOT, "tests", "cmake"), "-B", str(build),
                          f"-DBBM_SRC={src}", "-DBBM_BACKBONE=hip", f"-DBBM_HIP_ROOT={ou.ROOT}",
                          "-DCMAKE_BUILD_TYPE=Release"], capture_output=True, text=True, timeout=300)
    assert cfg.returncode == 0, cfg.stdout[-3000:] + cfg.stderr[-3000:]
    assert "Importing Backbone: hip" in cfg.stdout and "Available configurations: floatRGB;doubleRGB" in cfg.stdout
    assert "consumer: BBM_NAME=bbm BBM_BACKBONE=hip" in cfg.stdout
    b = subprocess.run(["cmake", "--build", str(build), "--target", "consumer", "-j", "4"], capture_output=True,
                       text=True, timeout=600)
    assert b.returncode == 0, b.stdout[-3000:] + b.stderr[-3000:]
    r = subprocess.run([str(build / "consumer")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d == {"abi": 12, "cooktorrance": "CookTorrance", "nested_children": 2, "failures": 0}
    # the configure step wrote its generated header into the copy, not into the reference
    assert (src / "include" / "bbm_bsdfmodels.h").exists()
