"""The device restatements of the host libm float functions the reference's native backbone calls (math.hpp:
expf_glibc, logf_glibc, powf_glibc, erff_glibc, erfcf_glibc) against the host libm of the machine running the test,
through bbm_hip_libm_eval: bit-identical floats (NaN = NaN) on strided sweeps of every float bit pattern and on
random (x, y) pairs for powf.  The C restatements of the same steps are pinned exhaustively on the CPU
(tests/test_oracle.py, oracle/*_check.c); this pins the device code to them."""
import ctypes

import numpy as np
import pytest

from tests import oracle_util as ou

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

FUNCS = {"expf": 0, "logf": 1, "powf": 2, "erff": 3, "erfcf": 4, "one_plus_sqrt": 5, "sinf": 6, "cosf": 7, "atan2f": 8, "theta": 9}


@pytest.fixture(scope="module")
def lib():
    import bbm_amd
    from bbm_amd import _lib
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return _lib.load()


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _device(lib, func, a, b=None):
    from bbm_amd import _lib
    da = torch.from_numpy(a).cuda()
    db = torch.from_numpy(b).cuda() if b is not None else None
    out = torch.empty_like(da)
    _lib.check(lib.bbm_hip_libm_eval(FUNCS[func], da.data_ptr(), db.data_ptr() if db is not None else None,
                                     out.data_ptr(), a.size, None))
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _host(func, a, b=None):
    out = np.empty_like(a)
    rc = ou.port().bbmport_libm(FUNCS[func], _fp(a), _fp(b) if b is not None else None, _fp(out),
                                ctypes.c_size_t(a.size))
    assert rc == 0
    return out


def _same(got, want):
    g, w = got.view(np.uint32), want.view(np.uint32)
    return (g == w) | (np.isnan(got) & np.isnan(want))


def _sweep(stride, offset=0):
    return (np.arange(offset, 1 << 32, stride, dtype=np.uint64)).astype(np.uint32).view(np.float32)


@pytest.mark.parametrize("func", ["expf", "logf", "erff", "erfcf"])
def test_unary_bitexact_sweep(lib, func):
    a = _sweep(251, 7)            # 17.1 M bit patterns: both signs, subnormals, inf, NaN
    got, want = _device(lib, func, a), _host(func, a)
    bad = np.nonzero(~_same(got, want))[0]
    assert bad.size == 0, f"{func}: {bad.size} lanes differ, e.g. x={a[bad[:4]]} got={got[bad[:4]]} libm={want[bad[:4]]}"


def test_powf_bitexact(lib):
    rng = np.random.default_rng(20261017)
    n = 1 << 22
    xs = [rng.integers(0, 0x7f800000, n, dtype=np.uint32).view(np.float32),       # any positive float
          rng.uniform(0, 4, n).astype(np.float32),                                  # Bagher (theta - theta0, k), (t, p)
          rng.uniform(0, 4, n).astype(np.float32),
          rng.integers(0, 0x00800000, n, dtype=np.uint32).view(np.float32)]         # subnormal x
    ys = [rng.uniform(-64, 64, n).astype(np.float32), rng.uniform(0, 64, n).astype(np.float32),
          rng.uniform(0, 2, n).astype(np.float32), rng.uniform(-2, 2, n).astype(np.float32)]
    specials = np.array([0, 0, 1, 1, np.inf, np.inf, np.nan, 2, 0.5], np.float32)
    specials_y = np.array([2, -2, 7.5, np.nan, 3, -3, 0, 0, np.inf], np.float32)
    a = np.concatenate(xs + [specials])
    b = np.concatenate(ys + [specials_y])
    got, want = _device(lib, "powf", a, b), _host("powf", a, b)
    bad = np.nonzero(~_same(got, want))[0]
    assert bad.size == 0, f"powf: {bad.size} lanes differ, e.g. x={a[bad[:4]]} y={b[bad[:4]]} got={got[bad[:4]]} libm={want[bad[:4]]}"


def test_one_plus_sqrt_bitexact(lib):
    """math.hpp f_one_plus_sqrt (the GGX G1 denominator float(1.0 + sqrt(1.0 + alpha^2 tan^2)), ggx.h:180-185) against
    the same IEEE double steps in numpy: a float rsq seed + one Newton step, with the exact sequence on lanes near a
    float rounding midpoint -- so every lane must be bit-identical, including those the fallback takes."""
    rng = np.random.default_rng(20261018)
    n = 1 << 22
    a = np.concatenate([rng.uniform(1e-4, 4, n).astype(np.float32),                 # alpha^2 (roughness^2 products)
                        np.ones(n, np.float32),
                        np.array([0, 1, 2, 3.5, 1e-30, 1e30, 1e30, np.inf, 1], np.float32)])
    b = np.concatenate([np.exp(rng.uniform(np.log(1e-9), np.log(1e9), n)).astype(np.float32),   # tan^2 theta
                        rng.integers(0, 0x7f000000, n, dtype=np.uint32).view(np.float32),       # any finite >= 0
                        np.array([0, 0, 1e-38, 0.25, 1e-30, 1e30, 3e38, 1, np.nan], np.float32)])
    got = _device(lib, "one_plus_sqrt", a, b)
    want = (1.0 + np.sqrt(1.0 + a.astype(np.float64) * b.astype(np.float64))).astype(np.float32)
    bad = np.nonzero(~_same(got, want))[0]
    assert bad.size == 0, f"{bad.size} lanes differ, e.g. a={a[bad[:4]]} b={b[bad[:4]]} got={got[bad[:4]]} want={want[bad[:4]]}"


@pytest.mark.parametrize("func", ["sinf", "cosf"])
def test_sincos_bitexact_sweep(lib, func):
    """sincosf_glibc on its exact domain |x| < 120 (every sampler angle): a strided sweep of both signs against the
    host's sinf / cosf; beyond it (and inf / NaN) the device library's sincosf: finite where the host's is, NaN where
    it is NaN."""
    u = np.arange(3, 0x42f00000, 97, dtype=np.uint32)
    a = np.concatenate([u, u | np.uint32(0x80000000)]).view(np.float32)
    got, want = _device(lib, func, a), _host(func, a)
    bad = np.nonzero(~_same(got, want))[0]
    assert bad.size == 0, f"{func}: {bad.size} lanes differ, e.g. x={a[bad[:4]]} got={got[bad[:4]]} libm={want[bad[:4]]}"
    big = np.array([120, -120, 1e4, 3e38, np.inf, -np.inf, np.nan], np.float32)
    gb, wb = _device(lib, func, big), _host(func, big)
    assert np.array_equal(np.isnan(gb), np.isnan(wb)) and np.allclose(gb[~np.isnan(wb)], wb[~np.isnan(wb)], atol=1e-6)


def test_atan2f_bitexact(lib):
    """atan2f_glibc (fdlibm's e_atan2f.c / s_atanf.c, the reference's spherical::phi) against the host's atan2f:
    unit-vector components, any finite floats, mixed magnitudes, and the zero / infinity / NaN combinations."""
    rng = np.random.default_rng(20261019)
    n = 1 << 22
    v = rng.normal(size=(3, n))
    v /= np.linalg.norm(v, axis=0)
    sp = np.array([0, -0.0, 1, -1, np.inf, -np.inf, np.nan, 1e-45, 3e38, 0.5], np.float32)
    ys = [v[1].astype(np.float32), rng.integers(0, 0xff800000, n, dtype=np.uint32).view(np.float32),
          (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-40, 40, n)).astype(np.float32), np.repeat(sp, sp.size)]
    xs = [v[0].astype(np.float32), rng.integers(0, 0xff800000, n, dtype=np.uint32).view(np.float32),
          (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-40, 40, n)).astype(np.float32), np.tile(sp, sp.size)]
    a, b = np.concatenate(ys), np.concatenate(xs)
    got, want = _device(lib, "atan2f", a, b), _host("atan2f", a, b)
    bad = np.nonzero(~_same(got, want))[0]
    assert bad.size == 0, f"{bad.size} lanes differ, e.g. y={a[bad[:4]]} x={b[bad[:4]]} got={got[bad[:4]]} libm={want[bad[:4]]}"


def test_theta_bitexact(lib):
    """theta_of (spectral.hpp: spherical::theta by a polynomial double asin with a midpoint guard) against numpy's
    IEEE double arcsin of the same float chord, rounded to float as the reference does: random unit and near-pole
    directions in both hemispheres, every lane bit-identical."""
    rng = np.random.default_rng(20261021)
    n = 1 << 22
    v = rng.normal(size=(2, n))
    v /= np.linalg.norm(v, axis=0)
    x = np.concatenate([v[0], rng.uniform(-1e-3, 1e-3, n // 4), [0, 1, -1, 0.70710678]]).astype(np.float32)
    z = np.concatenate([v[1], np.sign(rng.uniform(-1, 1, n // 4)) * np.sqrt(1 - 1e-6), [1, 0, 0, 0.70710678]]).astype(np.float32)
    got = _device(lib, "theta", x, z)
    f = np.float32
    sz = np.where(z < 0, f(-1), f(1))
    dz = (z - sz).astype(f)
    nrm = np.sqrt(((f(0) + x * x) + f(0) * f(0)) + dz * dz).astype(f)
    te = 2.0 * np.arcsin(0.5 * nrm.astype(np.float64))
    want = np.where(z >= 0, te, np.float64(np.float32(np.pi)) - te).astype(f)
    bad = np.nonzero(~_same(got, want))[0]
    assert bad.size == 0, f"{bad.size} lanes differ, e.g. x={x[bad[:4]]} z={z[bad[:4]]} got={got[bad[:4]]} want={want[bad[:4]]}"


CHUNK = 1 << 28
# |x| < 120 for the sin / cos restatement (every float the reference's cossin reaches)
SINCOS_HI = int(np.float32(120.0).view(np.uint32))
EXHAUSTIVE = {"expf": [(0, 1 << 32)], "logf": [(0, 1 << 32)], "erff": [(0, 1 << 32)], "erfcf": [(0, 1 << 32)],
              "sinf": [(0, SINCOS_HI), (1 << 31, (1 << 31) + SINCOS_HI)],
              "cosf": [(0, SINCOS_HI), (1 << 31, (1 << 31) + SINCOS_HI)]}


@pytest.mark.parametrize("func", list(EXHAUSTIVE))
def test_device_libm_exhaustive(lib, func):
    """Every float bit pattern (sinf / cosf: every |x| < 120) through the SHIPPED device code (bbm_hip_libm_eval ->
    math.hpp) against this machine's libm, bit for bit (NaN = NaN): the device restatements are pinned exhaustively
    themselves, not through a host transcription.  2^28 patterns per launch; the host side compares with OpenMP
    (oracle/port: bbmport_libm_sweep)."""
    from bbm_amd import _lib
    port = ou.port()
    port.bbmport_libm_sweep.restype = ctypes.c_longlong
    total, nbad, bad = 0, 0, []
    out = torch.empty(CHUNK, dtype=torch.float32, device="cuda")
    buf = np.empty(CHUNK, np.float32)
    badbuf = np.zeros(16, np.uint32)
    for lo, hi in EXHAUSTIVE[func]:
        for start in range(lo, hi, CHUNK):
            n = min(CHUNK, hi - start)
            bits = torch.arange(start, start + n, dtype=torch.int64, device="cuda")
            bits = torch.where(bits >= (1 << 31), bits - (1 << 32), bits).to(torch.int32)
            x = bits.view(torch.float32)
            _lib.check(lib.bbm_hip_libm_eval(FUNCS[func], x.data_ptr(), None, out.data_ptr(), n, None))
            torch.cuda.synchronize()
            buf[:n] = out[:n].cpu().numpy()
            k = port.bbmport_libm_sweep(FUNCS[func], ctypes.c_uint32(start), ctypes.c_size_t(n),
                                        buf.ctypes.data_as(ctypes.c_void_p), badbuf.ctypes.data_as(ctypes.c_void_p),
                                        16, 16)
            if k and len(bad) < 16:
                bad += [hex(int(b)) for b in badbuf[:min(k, 16)]]
            nbad += k
            total += n
            del bits, x
        print(f"{func}: [{lo:#x}, {hi:#x}) swept", flush=True)
    print(f"{func}: {total} patterns, {nbad} differ from the host libm", flush=True)
    assert nbad == 0, f"{func}: {nbad} of {total} patterns differ, e.g. {bad}"
