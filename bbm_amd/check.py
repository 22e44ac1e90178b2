"""checkBsdf on the GPU -- the reference's BSDF validation driver (bin/checkBsdf.cpp) with every
statistic computed by one batched reduction kernel (bbm_hip_check) instead of a serial loop.

    python -m bbm_amd.check bsdfmodel="CookTorrance(roughness=0.3)" test=reflectance samples=1000000 theta=4
    (torchrun ... -m bbm_amd.check ...  shards the samples over the GPUs of a node)

Tests, options and printed lines follow checkBsdf.cpp:420-479 (`test=` reflectance | reciprocity |
adjoint | pdf | pdfInt | sample; options as `key=value`, a bare `key` meaning true,
include/util/option.h).  Each test also returns its numbers as a dict.

Differences from the reference, by design:
  * random numbers: a counter-based generator with one stream per (test, slot, draw)
    (bbm_hip_check_draws) replaces the single std::mt19937 -- results are statistically equivalent,
    and identical whatever the number of GPUs (each rank draws its shard's numbers itself);
  * sums are accumulated in double (the reference accumulates floats serially);
  * the pdf test does not stop early at maxError failures and does not print each failure: it
    reports the counts (maxError is accepted for compatibility).
Multi-GPU: samples are split into contiguous shards (bbm_amd.fit.shard_range); per-rank
accumulators are gathered with torch.distributed and merged (sums add, maxima keep the largest value
with the lowest sample index) -- one tiny collective per test.
"""
import ctypes
import math
import sys

import numpy as np

from . import _lib
from .backbone import AggregateModel, BsdfModel, _stream_ptr, _torch, fromString, tree_desc

REFLECTANCE, RECIPROCITY, ADJOINT, PDF, PDFINT, SAMPLE_PDF, SAMPLE_COUNT = range(7)
ACC = 12
NSUMS = 8
DEFAULT_SEED = 5489                 # std::mt19937's default seed (the reference never seeds `rnd`)
EPSILON = float(np.finfo(np.float32).eps)
_F32 = np.float32
PI = _F32(math.pi)


class CheckDesc(ctypes.Structure):
    """bbm_hip_check_desc (include/bbm_hip.h)."""
    _fields_ = [("test", ctypes.c_int32), ("nslots", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("begin", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("slot_x", ctypes.c_void_p), ("slot_y", ctypes.c_void_p), ("slot_z", ctypes.c_void_p),
                ("sphere", ctypes.c_int32), ("importance", ctypes.c_int32), ("include_zero_pdf", ctypes.c_int32),
                ("theta_bins", ctypes.c_uint32), ("phi_bins", ctypes.c_uint32)]


def shard_range(total, rank, world):
    q, r = divmod(int(total), int(world))
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def merge_acc(parts):
    """Merge per-shard accumulators (nslots, ACC): sums add; (max, index) pairs keep the larger
    value, the lower sample index on ties (the serial loop keeps the first strict maximum)."""
    parts = [np.asarray(p, np.float64) for p in parts]
    out = parts[0].copy()
    for p in parts[1:]:
        out[:, :NSUMS] += p[:, :NSUMS]
        for m in (NSUMS, NSUMS + 2):
            take = (p[:, m] > out[:, m]) | ((p[:, m] == out[:, m]) & (p[:, m + 1] < out[:, m + 1]))
            out[take, m] = p[take, m]
            out[take, m + 1] = p[take, m + 1]
    return out


def _rank_world(dist):
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _gather_acc(acc, dist):
    """All ranks' accumulators -> merged (identical on every rank)."""
    rank, world = _rank_world(dist)
    if world == 1:
        return acc
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(acc)).to(dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return merge_acc([p.cpu().numpy() for p in parts])


def _sum_counts(counts, dist):
    rank, world = _rank_world(dist)
    if world == 1:
        return counts
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(counts.astype(np.int64))).to(dev)
    dist.all_reduce(t)
    return t.cpu().numpy()


def run(model, test, samples, nslots=1, slot_dirs=None, seed=DEFAULT_SEED, sphere=False, importance=False,
        include_zero=False, bins=(0, 0), begin=0, stream=None, f64=False):
    """One checkBsdf statistic over samples [begin, begin + samples) of every slot on this GPU: a single floatRGB
    model through its fused reduction kernel (bbm_hip_check); any other model (composed / runtime aggregates) or
    the doubleRGB configuration (f64) through the materialised path (bbm_hip_check_tree / _f64).
    Returns the (nslots, ACC) float64 accumulators, or for SAMPLE_COUNT the (nslots, bins) counts."""
    torch = _torch()
    lib = _lib.load()
    dev = torch.device("cuda", torch.cuda.current_device())
    tree = bool(f64) or isinstance(model, AggregateModel)
    d = CheckDesc()
    d.test, d.nslots, d.seed, d.begin, d.n = int(test), int(nslots), int(seed), int(begin), int(samples)
    keep = None
    sptr = (None, None, None)
    if slot_dirs is not None:
        keep = slot_dirs.to(dev, torch.float64 if f64 else torch.float32).contiguous()
        sptr = (keep[0].data_ptr(), keep[1].data_ptr(), keep[2].data_ptr())
        if not f64:
            d.slot_x, d.slot_y, d.slot_z = sptr
    d.sphere, d.importance, d.include_zero_pdf = int(bool(sphere)), int(bool(importance)), int(bool(include_zero))
    d.theta_bins, d.phi_bins = int(bins[0]), int(bins[1])
    nb = int(bins[0]) * int(bins[1])
    if test == SAMPLE_COUNT:
        out = torch.empty((nslots, nb), dtype=torch.int64, device=dev)
        acc_ptr, cnt_ptr = None, out.data_ptr()
        ws, wsb = None, 0
    else:
        out = torch.empty((nslots, ACC), dtype=torch.float64, device=dev)
        acc_ptr, cnt_ptr = out.data_ptr(), None
        wsf = lib.bbm_hip_check_tree_workspace_size if tree else lib.bbm_hip_check_workspace_size
        wsb = int(wsf(ctypes.byref(d)))
        wst = torch.empty(max(wsb // 8, 1), dtype=torch.float64, device=dev)
        ws = wst.data_ptr()
    if tree:
        desc, ndesc, _kd = tree_desc(model, bool(f64))
        if f64:
            _lib.check(lib.bbm_hip_check_tree_f64(desc, ndesc, ctypes.byref(d), sptr[0], sptr[1], sptr[2], acc_ptr,
                                                  cnt_ptr, ws, wsb, _stream_ptr(stream)))
        else:
            _lib.check(lib.bbm_hip_check_tree(desc, ndesc, ctypes.byref(d), acc_ptr, cnt_ptr, ws, wsb,
                                              _stream_ptr(stream)))
    else:
        _lib.check(lib.bbm_hip_check(model.model_id, model._pptr(), model._params.size, ctypes.byref(d), acc_ptr,
                                     cnt_ptr, ws, wsb, _stream_ptr(stream)))
    res = out.cpu().numpy()
    del keep
    return res


def draws(test, seed, slot, draw, offset, n, stream=None):
    """The uniforms (xi0, xi1) draw `draw` of `slot` uses for samples offset .. offset + n - 1."""
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device())
    u = torch.empty((2, n), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().bbm_hip_check_draws(int(test), int(seed), int(slot), int(draw), int(offset), int(n),
                                               u[0].data_ptr(), u[1].data_ptr(), _stream_ptr(stream)))
    return u


def trial_directions(test, seed, ntrials, sphere=False, stream=None):
    """The trial directions of pdfInt / sample (checkBsdf.cpp:270, :322) -> (3, ntrials) CUDA tensor."""
    torch = _torch()
    dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.empty((3, ntrials), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().bbm_hip_check_trials(int(test), int(seed), int(ntrials), int(bool(sphere)), t[0].data_ptr(),
                                                t[1].data_ptr(), t[2].data_ptr(), _stream_ptr(stream)))
    return t


def reflectance_outs(numtheta):
    """out directions of the reflectance test (checkBsdf.cpp:73-76): theta = idx Pi(0.5) / numtheta, phi = 0."""
    idx = np.arange(numtheta)
    theta = (idx.astype(_F32) * _F32(0.5 * math.pi)) / _F32(numtheta)
    st = np.sin(theta.astype(np.float64)).astype(_F32)
    ct = np.cos(theta.astype(np.float64)).astype(_F32)
    return np.stack([_F32(1.0) * st, _F32(0.0) * st, ct]).astype(_F32)


def _fmt(v):
    return "[" + ", ".join(f"{float(x):g}" for x in np.ravel(v)) + "]"


def _say(verbose, *a):
    if verbose:
        print(*a, flush=True)


# ------------------------------------------------------------------------------------ tests

def test_reflectance(bsdf, samples=100000, theta=1, importanceSampling=False, seed=DEFAULT_SEED, dist=None,
                     verbose=True):
    """checkBsdf.cpp:51-97: MC estimate of the reflectance per theta_out vs bsdf.reflectance(out)."""
    torch = _torch()
    rank, world = _rank_world(dist)
    b, e = shard_range(samples, rank, world)
    outs = reflectance_outs(theta)
    dout = torch.from_numpy(outs).cuda()
    acc = run(bsdf, REFLECTANCE, e - b, theta, dout, seed, importance=importanceSampling, begin=b)
    acc = _gather_acc(acc, dist)
    est = (acc[:, :3] / float(samples)).astype(np.float32)
    refl = bsdf.reflectance(dout).cpu().numpy().T
    _say(verbose and rank == 0, f"Reflectance test with {theta} directions and {samples} samples.")
    for t in range(theta):
        _say(verbose and rank == 0, f" out = {_fmt(outs[:, t])} => Estimate: {_fmt(est[t])} vs. {_fmt(refl[t])}")
    return {"out": outs.T, "estimate": est, "reflectance": refl, "accepted": acc[:, 3], "acc": acc}


def test_reciprocity(bsdf, samples=1000000, seed=DEFAULT_SEED, dist=None, verbose=True):
    """checkBsdf.cpp:102-140: average / max |f(in, out) - f(out, in)| over random sphere pairs."""
    return _symmetry(bsdf, RECIPROCITY, samples, seed, dist, verbose)


def test_adjoint(bsdf, samples=100000, seed=DEFAULT_SEED, dist=None, verbose=True):
    """checkBsdf.cpp:145-185: average / max |f_Radiance(in, out) - f_Importance(out, in)|."""
    return _symmetry(bsdf, ADJOINT, samples, seed, dist, verbose)


def _pair_at(test, seed, index):
    """The (in, out) sphere pair of sample `index` (draws 0 and 1 of slot 0)."""
    torch = _torch()
    lib = _lib.load()
    res = []
    for draw in (0, 1):
        u = draws(test, seed, 0, draw, index, 1)
        d = torch.empty((3, 1), dtype=torch.float32, device=u.device)
        _lib.check(lib.bbm_hip_sphere_dirs(u[0].data_ptr(), u[1].data_ptr(), 1, 0, d[0].data_ptr(), d[1].data_ptr(),
                                           d[2].data_ptr(), _stream_ptr(None)))
        res.append(d)
    return res


def _symmetry(bsdf, test, samples, seed, dist, verbose):
    rank, world = _rank_world(dist)
    b, e = shard_range(samples, rank, world)
    acc = _gather_acc(run(bsdf, test, e - b, 1, None, seed, begin=b), dist)[0]
    res = {"acc": acc}
    for tag, off, m in (("radiance", 0, NSUMS), ("importance", 3, NSUMS + 2)):
        if test == ADJOINT and tag == "importance":
            break
        avg = (acc[off:off + 3] / float(samples)).astype(np.float32)
        maxv, idx = acc[m], int(acc[m + 1])
        if samples > 0 and maxv > 0:
            din, dout = _pair_at(test, seed, idx)
            f1 = bsdf.eval(din, dout).cpu().numpy()[:, 0]
            f2 = bsdf.eval(dout, din).cpu().numpy()[:, 0]
            pair = (din.cpu().numpy()[:, 0], dout.cpu().numpy()[:, 0])
            maxd = np.abs(f1 - f2)
        else:
            idx, pair, maxd = -1, (np.zeros(3, _F32), np.zeros(3, _F32)), np.zeros(3, _F32)
        res[tag] = {"average": avg, "max": maxd, "max_hsum": max(maxv, 0.0), "at": pair, "sample": idx}
    if rank == 0 and verbose:
        if test == RECIPROCITY:
            for tag, label in (("radiance", "Radiance  "), ("importance", "Importance")):
                r = res[tag]
                print(f"{label} average = {_fmt(r['average'])}, max = {_fmt(r['max'])} at "
                      f"{{{_fmt(r['at'][0])}, {_fmt(r['at'][1])}}}", flush=True)
        else:
            r = res["radiance"]
            print(f"Adjoint difference average = {_fmt(r['average'])}, max = {_fmt(r['max'])} at "
                  f"{{{_fmt(r['at'][0])}, {_fmt(r['at'][1])}}}", flush=True)
    return res


def test_pdf(bsdf, samples=100000, maxError=10, checkBelowHorizon=False, sampleSphere=False, seed=DEFAULT_SEED,
             dist=None, verbose=True):
    """checkBsdf.cpp:190-245: pdf >= 0 and sample().pdf == pdf(sample().direction, out)."""
    rank, world = _rank_world(dist)
    b, e = shard_range(samples, rank, world)
    acc = _gather_acc(run(bsdf, PDF, e - b, 1, None, seed, sphere=sampleSphere, begin=b), dist)[0]
    res = {"negative": (int(acc[0]), int(acc[1])), "below_horizon": (int(acc[2]), int(acc[3])),
           "mismatch": (float(np.float32(acc[4] / samples)), float(np.float32(acc[5] / samples))), "acc": acc}
    if rank == 0 and verbose:
        line = f"PDF has {res['negative'][0]}/{res['negative'][1]} negative PDF values, "
        if checkBelowHorizon:
            line += f"{res['below_horizon'][0]}/{res['below_horizon'][1]} sampled directions below the horizon, "
        line += (f"and {res['mismatch'][0]:g}/{res['mismatch'][1]:g} average difference between the PDF from the "
                 "sample method and the corresponding PDF from the pdf-method.")
        print(f"Tesing PDF properties test with {samples} samples.", flush=True)
        print(line, flush=True)
    return res


def test_pdf_int(bsdf, samples=1000000, trials=10, sampleSphere=False, seed=DEFAULT_SEED, dist=None, verbose=True):
    """checkBsdf.cpp:250-290: MC integral of pdf(., t) over the sphere for `trials` directions t."""
    rank, world = _rank_world(dist)
    b, e = shard_range(samples, rank, world)
    t = trial_directions(PDFINT, seed, trials, sampleSphere)
    acc = _gather_acc(run(bsdf, PDFINT, e - b, trials, t, seed, begin=b), dist)
    integ = (acc[:, :2] / float(samples)).astype(np.float32)
    tn = t.cpu().numpy()
    if rank == 0 and verbose:
        print(f"Tesing PDF Integral with {samples} samples, for {trials} random directions sampled over the "
              f"{'sphere' if sampleSphere else 'hemisphere'}", flush=True)
        for k in range(trials):
            print(f" Integral = {integ[k, 0]:g}/{integ[k, 1]:g} (radiance/importance) for {_fmt(tn[:, k])}", flush=True)
    return {"integral": integ, "directions": tn.T, "acc": acc}


def gamma_q(a, x):
    """Regularised upper incomplete gamma Q(a, x) (include/util/gamma.h:564): series for x < a + 1,
    Legendre continued fraction otherwise (Numerical Recipes 6.2), in double."""
    a, x = float(a), float(x)
    if x < 0 or a <= 0:
        return 0.0
    if x == 0:
        return 1.0
    lg = math.lgamma(a)
    if x < a + 1:
        ap, s, term = a, 1.0 / a, 1.0 / a
        for _ in range(10000):
            ap += 1
            term *= x / ap
            s += term
            if abs(term) < abs(s) * 1e-16:
                break
        return max(0.0, 1.0 - s * math.exp(-x + a * math.log(x) - lg))
    tiny = 1e-300
    b = x + 1 - a
    c, d = 1 / tiny, 1 / b
    h = d
    for k in range(1, 10000):
        an = -k * (k - a)
        b += 2
        d = an * d + b
        d = tiny if abs(d) < tiny else d
        c = b + an / c
        c = tiny if abs(c) < tiny else c
        d = 1 / d
        delta = d * c
        h *= delta
        if abs(delta - 1) < 1e-16:
            break
    return math.exp(-x + a * math.log(x) - lg) * h


def chi2(pdf_bins, counts, samples):
    """checkBsdf.cpp:384-397: chi-square of the sample histogram against the integrated pdf."""
    m = pdf_bins.astype(np.float64) * samples
    ok = (m > EPSILON) & (counts > 5)
    c2 = float(np.sum((counts[ok] - m[ok]) ** 2 / m[ok]))
    df = int(ok.sum()) - 1
    return c2, df


def test_sample(bsdf, pdfSamples=4096, samples=100000, theta=10, phi=20, trials=10, sampleSphere=False,
                includeZeroPdfSamples=False, seed=DEFAULT_SEED, dist=None, verbose=True):
    """checkBsdf.cpp:295-418: chi-square test of sample() against pdf() over (theta x phi) bins."""
    rank, world = _rank_world(dist)
    bins = theta * phi
    t = trial_directions(SAMPLE_COUNT, seed, trials, sampleSphere)
    pb, pe = shard_range(pdfSamples, rank, world)
    acc = _gather_acc(run(bsdf, SAMPLE_PDF, pe - pb, trials * bins, t, seed, bins=(theta, phi), begin=pb), dist)
    pdf = (acc[:, 0] / float(pdfSamples)).reshape(trials, bins)
    sb, se = shard_range(samples, rank, world)
    counts = _sum_counts(run(bsdf, SAMPLE_COUNT, se - sb, trials, t, seed, bins=(theta, phi), begin=sb,
                             include_zero=includeZeroPdfSamples), dist)
    tn = t.cpu().numpy()
    out = []
    if rank == 0 and verbose:
        line = (f"Testing if sample and pdf match: {pdfSamples} PDF samples per bin, and {samples} direction samples, "
                f"with ({phi} x {theta}) bins over {trials} trials")
        if includeZeroPdfSamples:
            line += ", including zero pdf samples"
        print(line + ".", flush=True)
    for k in range(trials):
        c2, df = chi2(pdf[k], counts[k], samples)
        P = gamma_q((df - 1) / 2, c2 / 2) if df > 1 else None
        out.append({"direction": tn[:, k], "chi2": c2, "df": df, "P": P})
        if rank == 0 and verbose:
            print(f" Chi2 for {_fmt(tn[:, k])} = {c2:g} (with {df} degrees of freedom).", flush=True)
            if P is not None:
                print(f"  P = {P:g} (reject if lower than confidence).", flush=True)
            else:
                print(" No degrees of freedom; need at least 1 to compute P.", flush=True)
    return {"trials": out, "pdf": pdf, "counts": counts}


# -------------------------------------------------------------------------------------- CLI

TESTS = {
    "reflectance": (test_reflectance, {"samples": int, "theta": int, "importanceSampling": bool}),
    "reciprocity": (test_reciprocity, {"samples": int}),
    "adjoint": (test_adjoint, {"samples": int}),
    "pdf": (test_pdf, {"samples": int, "maxError": int, "checkBelowHorizon": bool, "sampleSphere": bool}),
    "pdfInt": (test_pdf_int, {"samples": int, "trials": int, "sampleSphere": bool}),
    "sample": (test_sample, {"pdfSamples": int, "samples": int, "theta": int, "phi": int, "trials": int,
                             "sampleSphere": bool, "includeZeroPdfSamples": bool}),
}


def parse_options(argv):
    """option_parser (include/util/option.h): `key=value`, or a bare `key` meaning true."""
    opt = {}
    for a in argv:
        if "=" in a:
            k, v = a.split("=", 1)
            opt[k.strip()] = v.strip()
        else:
            opt[a.strip()] = "true"
    return opt


def _convert(v, typ):
    if typ is bool:
        return v.lower() in ("1", "true", "yes", "on")
    return typ(v)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print("Usage: python -m bbm_amd.check [bsdfmodel=<bsdf string>] [test=<test name> [test options]]")
        for name, (_, keys) in TESTS.items():
            print(f"  + test={name} " + " ".join(f"[{k}]" for k in keys))
        return -1
    opt = parse_options(argv)
    model = opt.pop("bsdfmodel", "")
    test = opt.pop("test", "")
    seed = int(opt.pop("seed", DEFAULT_SEED))
    if test == "":
        print("ERROR: no test specified.")
        return -1
    if test not in TESTS:
        print(f"Unrecognized test: '{test}'")
        return 0
    fn, keys = TESTS[test]
    invalid = [k for k in opt if k not in keys]
    if invalid:
        print(f"ERROR: invalid keywords: {invalid}.")
        return 0
    import os
    torch = _torch()
    dist = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    bsdf = fromString(model) if model else BsdfModel("Lambertian")
    fn(bsdf, seed=seed, dist=dist, **{k: _convert(v, keys[k]) for k, v in opt.items()})
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
