"""Merl (include/staticmodel/merl.h) on the CPU side: the oracle pinned against the reference's own
import + lookup, the MERL file format, and the C-ABI's argument checks (no GPU compute).

No measured MERL file ships with the reference, so the data is synthetic (tests/oracle_util.synthetic_merl)
written in the MERL-MIT .binary format; the reference itself (oracle/_ref, its own merl_data) reads it.
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_util as ou

needs_ref = pytest.mark.skipif(ou.ref() is None, reason="oracle/_ref not built")


@pytest.fixture(scope="module")
def merl_file(tmp_path_factory):
    path = tmp_path_factory.mktemp("merl") / "synthetic.binary"
    raw = ou.synthetic_merl(path)
    return path, raw


@needs_ref
def test_reference_eval_is_white_balanced_table_at_linearizer_index(merl_file):
    """merl_data::eval (merl.h:78-96) == table[merl_linearizer(in, out)] with the import's white balance
    (merl.h:199-203): pins merl_table_numpy, the formula the GPU table builder restates."""
    path, raw = merl_file
    n = 200_000
    din = ou.dirgen_numpy(7, 0, 0, n, mode=1)
    dout = ou.dirgen_numpy(7, 1, 0, n, mode=1)
    ref = ou.ref_merl_eval_pdf(path, din, dout)
    idx = ou.ref_merl_index(din, dout).astype(np.int64)
    table = ou.merl_table_numpy(raw)
    above = (din[2] >= 0) & (dout[2] >= 0)
    want = np.zeros((3, n), np.float32)
    want[:, above] = table[:, idx[above]]
    np.testing.assert_array_equal(ref[:3], want)
    assert (table == 0).mean() > 0.015          # the -1 entries were clamped to 0


@needs_ref
def test_reference_string_form(merl_file):
    path, _ = merl_file
    assert ou.ref_merl_to_string(path) == f"Merl(\"{path}\")"


@needs_ref
def test_file_errors_match_reference(tmp_path):
    from bbm_amd.merl import read_binary
    missing = tmp_path / "missing.binary"
    with pytest.raises(RuntimeError, match="unable to open MERL BRDF"):
        read_binary(missing)
    bad = tmp_path / "bad.binary"
    np.asarray([90, 90, 90], dtype="<u4").tofile(bad)
    with pytest.raises(RuntimeError, match="not a recognized MERL BRDF"):
        read_binary(bad)
    one = np.zeros((3, 2), np.float32)
    for p in (missing, bad):
        with pytest.raises(RuntimeError):
            ou.ref_merl_eval_pdf(p, one, one)
    short = tmp_path / "short.binary"
    np.asarray([90, 90, 180], dtype="<u4").tofile(short)
    with pytest.raises(RuntimeError, match="truncated"):
        read_binary(short)


def test_write_read_round_trip(tmp_path):
    from bbm_amd.merl import read_binary, write_binary
    rgb = np.random.default_rng(1).normal(size=(3, 90, 90, 180))
    write_binary(tmp_path / "x.binary", rgb)
    dims, raw = read_binary(tmp_path / "x.binary")
    assert dims == (90, 90, 180)
    np.testing.assert_array_equal(raw, rgb.reshape(-1))


def test_abi_merl_table_rejects_bad_arguments():
    from bbm_amd import _lib
    lib = _lib.load()
    buf = ctypes.c_void_p(1)       # never dereferenced: the checks come first
    assert lib.bbm_hip_merl_table(None, 90, 90, 180, buf, None) == _lib.ERR_INVALID_ARG
    assert lib.bbm_hip_merl_table(buf, 90, 90, 90, buf, None) == _lib.ERR_INVALID_ARG
    assert b"not a recognized MERL BRDF" in lib.bbm_hip_last_error()
    mid = lib.bbm_hip_model_id(b"Merl")
    assert mid >= 0 and lib.bbm_hip_model_nparams(mid) == 2
