"""TEST INFRASTRUCTURE: checkBsdf statistics (bin/checkBsdf.cpp:51-418) recomputed on the CPU by the
reference itself (oracle/_ref shim: model eval / pdf / sample, sampleSphere, chi-square binning,
gamma_q) from the SAME random draws as the GPU kernel (bbm_hip_check), so that every GPU statistic
can be compared number for number.

The counter-based draws are restated here in numpy (integer arithmetic, exact): `draws()` must equal
bbm_hip_check_draws bit for bit (checked on the GPU by tests/test_gpu_check.py).  Sums are taken in
float64 over float32 per-sample terms, like the GPU kernel.
"""
import ctypes

import numpy as np

from tests import oracle_util as ou

M64 = (1 << 64) - 1
REFLECTANCE, RECIPROCITY, ADJOINT, PDF, PDFINT, SAMPLE_PDF, SAMPLE_COUNT = range(7)
EPS = np.float32(np.finfo(np.float32).eps)


def _mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def _key(seed, test, draw, slot):
    """check_base_key + check_key (bbm_amd/csrc/bbm_hip.hip, check.hpp)."""
    base = int(_mix64(np.uint64(seed & M64))) ^ ((0xd1b54a32d192ed03 * (0x10000 * (test + 1) + draw + 1)) & M64)
    return int(_mix64(np.uint64((base + 0x2545f4914f6cdd1d * slot) & M64)))


def draws(test, seed, slot, draw, offset, n):
    """(2, n) float32 uniforms of rndVec2d() draw `draw` for samples offset .. offset + n - 1."""
    key = _key(seed, test, draw, slot)
    idx = np.arange(offset, offset + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _mix64(np.uint64(key) + np.uint64(0x9e3779b97f4a7c15) * idx)
    u0 = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    u1 = ((h >> np.uint64(16)) & np.uint64(0xffffff)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return np.stack([u0, u1])


def sphere_dirs(xi, hemisphere=False):
    """sampleSphere / sampleHemisphere (checkBsdf.cpp:28-45) by the reference: (3, n) dirs, (n,) pdf."""
    lib = ou.ref()
    xi = np.ascontiguousarray(xi, np.float32)
    n = xi.shape[1]
    d = np.zeros((3, n), np.float32)
    p = np.zeros(n, np.float32)
    lib.bbmref_sphere_dirs(ctypes.c_size_t(n), ou._fp(xi[0]), ou._fp(xi[1]), int(hemisphere), ou._fp(d[0]),
                           ou._fp(d[1]), ou._fp(d[2]), ou._fp(p))
    return d, p


def trial_dirs(test, seed, ntrials, sphere=False):
    """bbm_hip_check_trials: trial t = sphere/hemisphere direction of draw 3 of slot t, sample 0."""
    xi = np.concatenate([draws(test, seed, t, 3, 0, 1) for t in range(ntrials)], axis=1)
    return sphere_dirs(xi, hemisphere=not sphere)[0]


def chi2_bins(d, theta, phi):
    lib = ou.ref()
    d = np.ascontiguousarray(d, np.float32)
    n = d.shape[1]
    idx = np.zeros(n, np.uint64)
    lib.bbmref_chi2_bins(ctypes.c_size_t(n), ou._fp(d[0]), ou._fp(d[1]), ou._fp(d[2]), ctypes.c_size_t(theta),
                         ctypes.c_size_t(phi), ou._fp(idx))
    return idx


def chi2_bin_points(t, p, rnd, theta, phi):
    lib = ou.ref()
    t = np.ascontiguousarray(t, np.uint32)
    p = np.ascontiguousarray(p, np.uint32)
    rnd = np.ascontiguousarray(rnd, np.float32)
    n = t.size
    d = np.zeros((3, n), np.float32)
    w = np.zeros(n, np.float32)
    lib.bbmref_chi2_bin_points(ctypes.c_size_t(n), ou._fp(t), ou._fp(p), ou._fp(rnd[0]), ou._fp(rnd[1]),
                               ctypes.c_size_t(theta), ctypes.c_size_t(phi), ou._fp(d[0]), ou._fp(d[1]), ou._fp(d[2]),
                               ou._fp(w))
    return d, w


def gamma_q(a, x):
    lib = ou.ref()
    lib.bbmref_gamma_q.restype = ctypes.c_double
    lib.bbmref_gamma_q.argtypes = [ctypes.c_float, ctypes.c_float]
    return float(lib.bbmref_gamma_q(a, x))


def _bcast(v, n):
    return np.ascontiguousarray(np.repeat(np.asarray(v, np.float32).reshape(3, 1), n, axis=1))


def _eval(name, params, din, dout):
    """eval + pdf of the reference model `name` at `params`; name may also be a runtime-aggregate tree
    (oracle_util.runtime_tree form: the reference's own aggregatebsdf of bsdf_ptrs), params then unused."""
    if isinstance(name, tuple):
        return ou.ref_runtime_eval_pdf(name, din, dout)
    return ou.ref_eval_pdf(name, params, din, dout, nthreads=8)


def _sample(name, params, out, xi):
    if isinstance(name, tuple):
        return ou.ref_runtime_sample(name, out, xi)
    return ou.ref_sample(name, params, out, xi, nthreads=8)


def reflectance(name, params, out, samples, seed, slot, importance, begin=0):
    """checkBsdf.cpp:77-90 for one theta_out: sums of eval(dir, out) z(dir) / pdf, accepted count."""
    xi = draws(REFLECTANCE, seed, slot, 0, begin, samples)
    outs = _bcast(out, samples)
    if importance:
        s, _ = _sample(name, params, outs, xi)
        d, pdf = s[:3], s[3]
    else:
        d, pdf = sphere_dirs(xi)
    f = _eval(name, params, d, outs)[:3]
    ok = pdf > EPS
    term = (f[:, ok] * d[2, ok]) / pdf[ok]
    return np.array([term[0].sum(dtype=np.float64), term[1].sum(dtype=np.float64), term[2].sum(dtype=np.float64),
                     float(ok.sum())])


def symmetry(name, params, samples, seed, test, begin=0):
    """checkBsdf.cpp:112-132: sum |f(in, out) - f(out, in)| per channel and the first strict max of hsum."""
    din, _ = sphere_dirs(draws(test, seed, 0, 0, begin, samples))
    dout, _ = sphere_dirs(draws(test, seed, 0, 1, begin, samples))
    f1 = _eval(name, params, din, dout)[:3]
    f2 = _eval(name, params, dout, din)[:3]
    diff = np.abs(f1 - f2)
    h = ((np.float32(0) + diff[0]) + diff[1]) + diff[2]
    k = int(np.argmax(h))
    return diff.sum(axis=1, dtype=np.float64), float(h[k]), begin + k


def pdf_test(name, params, samples, seed, sphere, begin=0):
    """checkBsdf.cpp:216-237: negative pdf, below horizon and |sample.pdf - pdf| (Radiance; Importance
    uses the third draw)."""
    out, _ = sphere_dirs(draws(PDF, seed, 0, 0, begin, samples), hemisphere=not sphere)
    res = []
    for draw in (1, 2):
        s, _ = _sample(name, params, out, draws(PDF, seed, 0, draw, begin, samples))
        p = _eval(name, params, s[:3], out)[3]
        res.append((int((p < 0).sum()), int((s[2] < 0).sum()), float(np.abs(s[3] - p).sum(dtype=np.float64))))
    return res


def pdf_int(name, params, t, samples, seed, slot, begin=0):
    """checkBsdf.cpp:276-283: sum pdf(dir, t) / (1 / 4 pi) over sphere samples."""
    d, sp = sphere_dirs(draws(PDFINT, seed, slot, 0, begin, samples))
    p = _eval(name, params, d, _bcast(t, samples))[3]
    return float((p / sp).sum(dtype=np.float64))


def sample_pdf(name, params, t, trial, bins, pdf_samples, seed, theta, phi):
    """checkBsdf.cpp:341-357: sum over the bin's pdf samples of pdf(dir, t) * w, for every bin."""
    res = np.zeros(bins)
    for b in range(bins):
        slot = trial * bins + b
        rnd = draws(SAMPLE_PDF, seed, slot, 0, 0, pdf_samples)
        d, w = chi2_bin_points(np.full(pdf_samples, b // phi), np.full(pdf_samples, b % phi), rnd, theta, phi)
        p = _eval(name, params, d, _bcast(t, pdf_samples))[3]
        res[b] = (p * w).sum(dtype=np.float64)
    return res


def sample_count(name, params, t, trial, samples, seed, theta, phi, include_zero=False):
    """checkBsdf.cpp:360-380: histogram of sampled directions over the (theta x phi) bins."""
    xi = draws(SAMPLE_COUNT, seed, trial, 0, 0, samples)
    s, _ = _sample(name, params, _bcast(t, samples), xi)
    ok = np.ones(samples, bool) if include_zero else (s[3] > EPS)
    idx = chi2_bins(s[:3, ok], theta, phi)
    return np.bincount(idx.astype(np.int64), minlength=theta * phi)
