"""Merl (include/staticmodel/merl.h:224-225) on the GPU against the reference's own merl model
(oracle/_ref: merl_data + ndf::sampler, reading the same synthetic MERL .binary file).

eval is a lookup: every lane must read the reference's own (theta_h, theta_d, phi_d) bin, bit-exact.  The GPU
decides the bin by a cheap evaluation with error bounds and, where a coordinate lies within its bound of a bin
edge, by the reference's own float arithmetic (merl.hpp merl_bin), so no lane may flip (MAX_FLIP_FRAC = 0; the
neighbour check below stays as the diagnostic for a lane that would).
pdf / sample are the data-driven backscatter sampler shared with the He family (tolerances as there).
"""
import numpy as np
import pytest

from tests import oracle_util as ou

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(ou.ref() is None, reason="oracle/_ref not built")]

MAX_FLIP_FRAC = 0.0


@pytest.fixture(scope="module")
def bbm():
    import bbm_amd
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return bbm_amd


@pytest.fixture(scope="module")
def merl(bbm, tmp_path_factory):
    path = tmp_path_factory.mktemp("merl") / "synthetic.binary"
    raw = ou.synthetic_merl(path)
    return path, raw, bbm.Merl(path)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def _edge_cases():
    """in == out (phi_d undefined), normal incidence, grazing (z = 0, included by merl's >= 0 test),
    mirror pairs, below-horizon lanes."""
    t = np.linspace(0, np.pi / 2, 19)
    p = np.linspace(0, 2 * np.pi, 13)
    T, P = np.meshgrid(t, p)
    v = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)]).reshape(3, -1).astype(np.float32)
    mirror = v * np.float32([[-1], [-1], [1]])
    down = v * np.float32([[1], [1], [-1]])
    din = np.concatenate([v, np.float32([[0], [0], [1]]) + 0 * v, v, v, down], 1)
    dout = np.concatenate([v, v, mirror, np.float32([[1], [0], [0]]) + 0 * v, v], 1)
    return din, dout


def _check_eval(got, ref, din, dout, raw):
    """bit-exact except rare bin-edge lanes, which must read a neighbouring bin of the reference's"""
    diff = np.nonzero(np.any(got != ref, axis=0))[0]
    assert diff.size <= MAX_FLIP_FRAC * got.shape[1], f"{diff.size} of {got.shape[1]} lanes differ"
    if diff.size:
        table = ou.merl_table_numpy(raw)
        idx = ou.ref_merl_index(din[:, diff], dout[:, diff]).astype(np.int64)
        th, td, pd = idx // 16200, (idx // 180) % 90, idx % 180
        ok = np.zeros(diff.size, bool)
        for a in (-1, 0, 1):
            for b in (-1, 0, 1):
                for c in (-1, 0, 1):
                    j = (np.clip(th + a, 0, 89) * 90 + np.clip(td + b, 0, 89)) * 180 + (pd + c) % 180
                    ok |= np.all(table[:, j] == got[:, diff], axis=0)
        assert ok.all(), f"lanes {diff[~ok][:5]} read no neighbouring bin"
    return diff.size


def test_eval_pdf_vs_reference(merl):
    path, raw, m = merl
    n = 1 << 20
    for mode in (0, 1):
        din = ou.dirgen_numpy(11, 0, 0, n, mode=mode)
        dout = ou.dirgen_numpy(11, 1, 0, n, mode=mode)
        ei, eo = _edge_cases()
        din, dout = np.concatenate([din, ei], 1), np.concatenate([dout, eo], 1)
        rgb, pdf = m.eval_pdf(_dev(din), _dev(dout))
        torch.cuda.synchronize()
        ref = ou.ref_merl_eval_pdf(path, din, dout)
        flips = _check_eval(rgb.cpu().numpy(), ref[:3], din, dout, raw)
        got_pdf = pdf.cpu().numpy()
        bad = ou.parity_violations(got_pdf[None], ref[3:])
        assert len(bad[0]) == 0, f"pdf: {len(bad[0])} lanes outside tolerance"
        assert np.array_equal(got_pdf == 0, ref[3] == 0)
        print(f"mode {mode}: {flips} eval bin-edge lanes of {din.shape[1]}")


def test_eval_component_and_unit(merl):
    path, raw, m = merl
    n = 4096
    din = ou.dirgen_numpy(3, 0, 0, n, mode=0)
    dout = ou.dirgen_numpy(3, 1, 0, n, mode=0)
    for component in (0, 1, 2, 3):
        for unit in (0, 1):
            rgb, pdf = m.eval_pdf(_dev(din), _dev(dout), component=component, unit=unit)
            torch.cuda.synchronize()
            ref = ou.ref_merl_eval_pdf(path, din, dout, component=component, unit=unit)
            _check_eval(rgb.cpu().numpy(), ref[:3], din, dout, raw)
            if component == 0:      # the reference's sampler CDF is 0/0 there; masked lanes are 0 on both sides
                assert np.all(pdf.cpu().numpy() == 0) or np.array_equal(np.isnan(pdf.cpu().numpy()), np.isnan(ref[3]))
            else:
                bad = ou.parity_violations(pdf.cpu().numpy()[None], ref[3:])
                assert len(bad[0]) == 0, (component, unit)


def test_sample_vs_reference(merl):
    path, raw, m = merl
    n = 1 << 16
    dout = ou.dirgen_numpy(5, 2, 0, n, mode=1)
    xi = np.random.default_rng(5).random((2, n), dtype=np.float32)
    s = m.sample(_dev(dout), _dev(xi))
    torch.cuda.synchronize()
    d, p, f = s.direction.cpu().numpy(), s.pdf.cpu().numpy(), s.flag.cpu().numpy().astype(np.uint32)
    ref, flag = ou.ref_merl_sample(path, dout, xi)
    assert np.array_equal(f, flag)
    derr = np.abs(d.astype(np.float64) - ref[:3]).max(0)
    # the 90-bin CDF sums agree to ~1e-6: an xi0 at a bin edge may pick the neighbouring bin (test_gpu_parity)
    assert np.mean(derr > 1e-3) <= 1e-3
    assert np.mean(derr > 1e-5) <= 0.005
    close = derr <= 1e-5
    bad = ou.parity_violations(p[None, close], ref[3:, close])
    assert len(bad[0]) == 0


def test_reflectance_placeholder(merl):
    _, _, m = merl
    out = _dev(ou.dirgen_numpy(9, 2, 0, 1000, mode=1))
    for component, want in ((3, 1.0), (2, 0.0), (1, 0.0), (0, 0.0)):      # is_set(c, All), util/flags.h:100-103
        r = m.reflectance(out, component=component)
        torch.cuda.synchronize()
        assert torch.all(r == want)


def test_string_round_trip_and_errors(bbm, merl, tmp_path):
    path, _, m = merl
    assert str(m) == ou.ref_merl_to_string(path)
    m2 = bbm.fromString(str(m))
    din = _dev(ou.dirgen_numpy(1, 0, 0, 2048))
    dout = _dev(ou.dirgen_numpy(1, 1, 0, 2048))
    assert torch.equal(m.eval(din, dout), m2.eval(din, dout))
    # a Merl parameter vector without a table fails loudly instead of dereferencing null
    empty = bbm.BsdfModel.__new__(bbm.BsdfModel)
    empty.name, empty.model_id, empty._params = "Merl", m.model_id, np.zeros(2, np.float32)
    with pytest.raises(RuntimeError, match="no table"):
        empty.eval(din, dout)
    bad = tmp_path / "bad.binary"
    np.asarray([90, 90, 90], dtype="<u4").tofile(bad)
    with pytest.raises(RuntimeError, match="not a recognized MERL BRDF"):
        bbm.Merl(bad)
