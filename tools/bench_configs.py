"""bench.py --workload models|sample|fit|f64: BASELINE.json configs 3-5 and the doubleRGB path (one JSON line each).

  models  (config 3) every single bsdfmodel's eval over 10M shared pairs per GPU, one launch per model
          (bbm_hip_eval).  Algorithmic bytes: 24 B in + 12 B RGB out = 36 B/pair (models that read only
          z: 8 + 12 = 20 B).  Per-model pairs/s and fraction of the 8 TB/s HBM roofline.  Merl (measured data,
          a synthetic MERL .binary) also gathers one 16 B table entry per pair from its 23 MB table, which
          the L2/MALL serve; the 36 B/pair figure leaves that gather out.
  sample  (config 4) importance-sample -> eval -> pdf Monte-Carlo loop (checkBsdf's reflectance test,
          bbm_hip_check REFLECTANCE with importance sampling) for the microfacet models CookTorrance and
          GGX: 125M samples per GPU (1B over 8 GPUs), 8 theta_out slots, reduced in-kernel to per-slot
          sums -- no HBM traffic per sample, so the kernel is VALU-bound: reported as samples/s.
  fit     (config 5) the fitting loss of one compass step: Aggregate(Lambertian, Bagher) against a Merl
          reference (a MERL .binary holding a perturbed Bagher fit, read through bbm_amd.Merl) on the MERL grid (90 x 90 x 180 = 1.458M pairs, sharded over the GPUs),
          2P = 36 probes in one bbm_hip_loss launch, plus the RCCL all-reduce of the 36 partial sums
          when N > 1 (strong scaling: the grid is fixed).  Reported as probe-pair evaluations/s.
  f64     the doubleRGB configuration (bbm_hip_eval_pdf_f64): --model's eval+pdf over --pairs f64 pairs per GPU, 80 B
          per pair algorithmic (48 B in + 32 B out), and every model with doubleRGB kernels over 10M shared pairs.
Timing follows bench.py: warmup, barrier + synchronize around K timed steps, max over ranks.

cpu_baseline (rank 0, N = 1, unless --no-cpu): the reference itself (oracle/_ref/libbbm_ref.so: the reference headers
compiled with the native floatRGB backbone, OpenMP over every CPU this process may use, as bench.py's headline leg) on a
bounded sample of the same workload, about --cpu-seconds of CPU work per line:
  models  every model's eval (mode eval only) over a sample of the same pairs, ~--cpu-seconds / #models each
  sample  the reference's own loop (bin/checkBsdf.cpp:78-84): bsdf.sample(out, xi) then bsdf.eval(dir, out) per sample
  fit     sampledlossfunction::operator()(idx) (include/bbm/sampledlossfunction.h:62-73) over every pair of the MERL
          grid, once per probe -- the reference evaluates the fitted and the reference model per sample each time
lambertian-cpu (config 1, bench.py): the native backbone's Lambertian eval over 1M pairs, no GPU.
"""
import ctypes
import json
import os
import tempfile
import time

import numpy as np
import torch

import bbm_amd
from bbm_amd import _lib, check, fit, merl
from bbm_amd.backbone import _stream_ptr
from tools import bench_harness as bh

SEED = 0xBB5EED
HBM_PEAK_GBS = 8000.0
Z_ONLY = {"Lambertian"}
# f32 vector peak (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs x one wave64 VALU instruction per 2 cycles x 2.4 GHz
# = 1.2288e12 wave-instructions/s = 78.6e12 lane-instructions/s = 157.3 TFLOP/s counting an FMA as 2 flops
VALU_PEAK_TFLOPS = 157.3
VALU_LANE_INSTR_PEAK = VALU_PEAK_TFLOPS * 1e12 / 2
PMC_VALU_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_valu.json")


def _subset(args, names):
    if not args.models:
        return list(names)
    want = [m.strip() for m in args.models.split(",") if m.strip()]
    return [m for m in names if m in want]


def valu_roofline(key, kernel_ms, units):
    """VALU roofline of one workload's dominant kernel: its VALU instructions per unit come from the committed
    counter summary (profiles/pmc_valu.json, tools/valu_roofline.py: SQ_INSTS_VALU x 64 lanes / units per
    dispatch, collected by tools/gpu_step.sh pmc:...), its time from this run's HIP events.  achieved = issued
    lane-instructions/s x 2 (an FMA's two flops: the unit the 157.3 TFLOP/s f32 vector peak is quoted in), so
    frac = the fraction of the chip's VALU issue slots this kernel fills (an upper bound on its FLOP fraction)."""
    entry = None
    if os.path.exists(PMC_VALU_FILE):
        try:
            with open(PMC_VALU_FILE) as f:
                entry = json.load(f).get("workloads", {}).get(key)
        except (OSError, ValueError):
            entry = None
    if not entry:
        return {"bound": "valu", "achieved": None, "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": None,
                "traffic": None, "kernel_ms": kernel_ms, "note": f"no VALU counter summary for {key}"}
    per_unit = entry["valu_lane_instr_per_unit"]
    lane_rate = per_unit * units / (kernel_ms * 1e-3)
    achieved = 2 * lane_rate / 1e12
    return {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / VALU_PEAK_TFLOPS, "traffic": None, "kernel": entry.get("kernel"),
            "kernel_ms": kernel_ms, "valu_instr_per_unit": per_unit,
            "valu_active_lane_frac": entry.get("valu_active_lane_frac"),
            "counters": f"profiles/pmc_valu.json[{key}] ({entry.get('source', '')})"}


def _timed(step, args, dist, stream):
    """tools/bench_harness.timed: warmup, settle, barrier + synchronize around K steps, slowest rank."""
    elapsed, kern_ms, _, _ = bh.timed(step, args, dist, stream)
    return elapsed, kern_ms


def _line(args, world, metric, value, unit, elapsed, config, extra):
    d = {"metric": metric, "value": value, "unit": unit, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
         "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "vs_baseline": None, "dtype": "f32",
         "data": "synthetic", "config": config}
    d.update(extra)
    print(json.dumps(d), flush=True)


GRAPH_REPS = 8


def _graph(launch, reps):
    """A CUDA(HIP) graph of `reps` calls of launch(stream), captured after one warm-up call (first-use host work
    such as EPD's table build happens there, outside the capture)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        launch(side)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream()
        for _ in range(reps):
            launch(s)
    torch.cuda.synchronize()
    return g


MODEL_SETS = 4


# ---------------------------------------------------------------- CPU baselines (the reference on the host)

def cpu_threads():
    """(threads, description): every CPU this process may use -- the affinity mask capped by the cgroup CPU quota
    (bench.py cpu_baseline)."""
    aff, phys, smt, quota, cpu_model = bh.cpu_topology()
    threads = aff if quota is None else max(1, min(aff, int(-(-quota // 1))))
    desc = (f"OpenMP {threads} threads = every CPU this process may use (affinity mask: {aff} threads on {phys} "
            f"physical cores x {smt} SMT{'' if quota is None else f'; cgroup CPU quota {quota:g} CPUs'}) on {cpu_model}")
    return threads, desc


def _cpu_lib():
    """(library, kind): the compiled reference (oracle/_ref) or, without it, the C restatement (oracle/port: the
    models it covers only)."""
    from tests import oracle_util as ou
    if ou.ref() is not None:
        return ou.ref_bench(), "reference"
    return None, "port"


def _fp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _timed_calls(call, budget_s):
    """call() once untimed, then repeatedly until budget_s has passed -> (calls, seconds)."""
    call()
    done, t0 = 0, time.perf_counter()
    while True:
        call()
        done += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            return done, el


def _ref_eval_call(lib, name, params, hin, hout, mode, threads, merl_path=None):
    """A closure running the reference's eval (mode 1) / eval+pdf (3) over the host SoA pairs into preallocated rows."""
    n = hin.shape[1]
    out = np.zeros((4, n), np.float32)
    p = np.ascontiguousarray(params, np.float32)
    args = (ctypes.c_size_t(n), _fp(hin[0]), _fp(hin[1]), _fp(hin[2]), _fp(hout[0]), _fp(hout[1]), _fp(hout[2]),
            ctypes.c_uint32(3), ctypes.c_uint32(0), mode, _fp(out[0]), _fp(out[1]), _fp(out[2]), _fp(out[3]), threads)
    if merl_path is not None:
        fn = lambda: lib.bbmref_merl_eval_pdf(merl_path.encode(), *args)          # noqa: E731
    else:
        fn = lambda: lib.bbmref_eval_pdf(name.encode(), _fp(p), p.size, *args)    # noqa: E731

    def call():
        if fn() != 0:
            raise KeyError(f"reference has no model {name}")
    return call


def cpu_models(names, din, dout, seconds, merl_path=None):
    """Config 3's CPU column: the reference's eval of every model over a sample of the benchmark's pairs, about
    seconds / len(names) each; per-model pairs/s and the whole set's rate (sum of pairs / sum of times)."""
    lib, kind = _cpu_lib()
    if lib is None:
        return None
    threads, tdesc = cpu_threads()
    n_base = min(din.shape[1], 1 << 18)
    per, tot_pairs, tot_s = {}, 0, 0.0
    budget = max(seconds / max(len(names), 1), 0.2)
    for name in names:
        if name == "Merl" and merl_path is None:
            continue
        n = min(din.shape[1], 1 << 21) if name == "Merl" else n_base   # amortise the shim's per-call file read
        hin = np.ascontiguousarray(din[:, :n].cpu().numpy())
        hout = np.ascontiguousarray(dout[:, :n].cpu().numpy())
        params = bbm_amd.BsdfModel(name).parameter_values() if name != "Merl" else None
        call = _ref_eval_call(lib, name, params, hin, hout, 1, threads, merl_path if name == "Merl" else None)
        calls, el = _timed_calls(call, budget)
        per[name] = {"pairs_per_s": calls * n / el, "sample_pairs": n, "calls": calls, "seconds": el}
        tot_pairs += calls * n
        tot_s += el
    return {"value": tot_pairs / tot_s, "unit": "pairs/s", "cores": threads, "kind": kind,
            "sample": f"eval (no pdf) of each of {len(per)} models over the first {n_base} pairs of the benchmark's "
                      f"operand set 0 (Merl: {min(din.shape[1], 1 << 21)} pairs, the shim reading the .binary per call), "
                      f"repeated for ~{budget:.2f} s per model; value = all pairs / all seconds; via oracle/_ref "
                      f"(reference headers, native floatRGB); {tdesc}",
            "per_model": per}


def cpu_sample(names, outs, slots, seconds):
    """Config 4's CPU column: the reference's importance-sampled reflectance loop (bin/checkBsdf.cpp:78-84: sample
    then eval at the sampled direction, accumulated where pdf > Epsilon) over a bounded sample per model."""
    lib, kind = _cpu_lib()
    if lib is None:
        return None
    threads, tdesc = cpu_threads()
    n = 1 << 20
    rng = np.random.default_rng(SEED)
    o = np.ascontiguousarray(np.repeat(outs.cpu().numpy(), n // slots, axis=1))
    xi = rng.random((2, n), dtype=np.float32)
    per = {}
    for name in names:
        p = np.ascontiguousarray(bbm_amd.BsdfModel(name).parameter_values(), np.float32)
        d = np.zeros((4, n), np.float32)
        flag = np.zeros(n, np.uint32)
        ev = np.zeros((4, n), np.float32)

        def call():
            rc = lib.bbmref_sample(name.encode(), _fp(p), p.size, ctypes.c_size_t(n), _fp(o[0]), _fp(o[1]), _fp(o[2]),
                                   _fp(xi[0]), _fp(xi[1]), ctypes.c_uint32(3), ctypes.c_uint32(0), _fp(d[0]), _fp(d[1]),
                                   _fp(d[2]), _fp(d[3]), _fp(flag), threads)
            assert rc == 0
            rc = lib.bbmref_eval_pdf(name.encode(), _fp(p), p.size, ctypes.c_size_t(n), _fp(d[0]), _fp(d[1]), _fp(d[2]),
                                     _fp(o[0]), _fp(o[1]), _fp(o[2]), ctypes.c_uint32(3), ctypes.c_uint32(0), 1,
                                     _fp(ev[0]), _fp(ev[1]), _fp(ev[2]), _fp(ev[3]), threads)
            assert rc == 0
            keep = d[3] > np.float32(np.finfo(np.float32).eps)
            (ev[:3, keep] * (d[2, keep] / d[3, keep])).sum(axis=1)
        calls, el = _timed_calls(call, seconds / max(len(names), 1))
        per[name] = {"samples_per_s": calls * n / el, "calls": calls, "seconds": el}
    head = next(iter(per))
    return {"value": per[head]["samples_per_s"], "unit": "samples/s", "cores": threads, "kind": kind,
            "sample": f"{n} samples per call ({slots} theta_out x {n // slots}, xi from numpy), the reference's "
                      f"sample -> eval -> z / pdf accumulation as checkBsdf's reflectance test, repeated for "
                      f"~{seconds / max(len(names), 1):.1f} s per model; value = {head}; via oracle/_ref; {tdesc}",
            "per_model": per}


def cpu_fit(name, fitted, reference, lin, seconds):
    """Config 5's CPU column: the reference's sampledlossfunction over the same MERL-grid pairs, one probe per call
    (operator()(idx) for every idx, OpenMP; each sample evaluates the fitted and the reference model, as the
    reference does), for about `seconds`."""
    lib, kind = _cpu_lib()
    if lib is None:
        return None
    from tests import oracle_util as ou
    threads, tdesc = cpu_threads()
    din, dout = lin.directions()
    hin, hout = din.cpu().numpy(), dout.cpu().numpy()
    fp = fitted.parameter_values()
    rp = reference.parameter_values()
    calls, el = _timed_calls(lambda: ou.ref_pair_losses(name, fp, rp, hin, hout, 3, nthreads=threads, lib=lib), seconds)
    n = hin.shape[1]
    return {"value": calls * n / el, "unit": "probe-pairs/s", "cores": threads, "kind": kind,
            "sample": f"{calls} probes x the {n} MERL-grid pairs (standardLog), reference = the analytic fit "
                      f"(fits/{FIT_MATERIAL[0]}:3), ~{seconds:.0f} s; the reference's sampledlossfunction evaluates "
                      f"both models per sample and probe; via oracle/_ref; {tdesc}"}


def bench_models(args, dist, rank, world):
    """Config 3.  Every model's eval over 10M pairs per GPU, timed as HIP-graph replays of GRAPH_REPS launches that
    cycle over MODEL_SETS distinct input/output sets (360 MB each, 1.44 GB in all): no launch finds its operands in
    the 256 MiB Infinity Cache left behind by the previous one, so the HBM fractions are HBM measurements."""
    n = 10_000_000
    sets = []
    for k in range(MODEL_SETS):
        sets.append((bbm_amd.fill_directions(SEED + k, 0, rank * n, n, mode=0),
                     bbm_amd.fill_directions(SEED + k, 1, rank * n, n, mode=0),
                     torch.empty((3, n), dtype=torch.float32, device="cuda")))
    stream = torch.cuda.current_stream()
    per = {}
    total_t = 0.0
    names = _subset(args, [m for m in bbm_amd.model_names() if not m.startswith("Aggregate")])
    reps = GRAPH_REPS
    for name in names:
        m = _merl_from(bbm_amd.CookTorrance()) if name == "Merl" else bbm_amd.BsdfModel(name)
        # one step = a HIP graph of `reps` back-to-back launches: a 10M-pair eval of the HBM-bound models takes
        # ~50 us, less than one Python-side launch, so per-launch stepping would time the host, not the kernel
        cyc = [0]

        def launch(s):
            din, dout, rgb = sets[cyc[0] % MODEL_SETS]
            cyc[0] += 1
            m.eval_pdf(din, dout, rgb=rgb, mode=1, stream=s)
        if args.graph == "off":
            # counter passes (rocprofv3 --pmc serialises dispatches): the same launches issued one by one
            step = lambda: [launch(stream) for _ in range(reps)]   # noqa: E731
        else:
            step = _graph(launch, reps).replay
        elapsed, step_ms = _timed(step, args, dist, stream)
        kern_ms = step_ms / reps
        bpp = 20 if name in Z_ONLY else 36
        gbs = bpp * n / (kern_ms * 1e-3) / 1e9
        per[name] = {"pairs_per_s": n * world * args.steps * reps / elapsed, "kernel_ms": kern_ms, "GB_s": gbs,
                     "roofline_frac": gbs / HBM_PEAK_GBS, "bytes_per_pair": bpp}
        if name == "Merl":
            # the table entry each pair reads is algorithmic data too (one float4 of the 23 MB table; random
            # directions touch a different cache line per pair, which the Infinity Cache serves)
            per[name]["with_table_gather"] = {"bytes_per_pair": 52,
                                              "roofline_frac": 52 * n / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        vr = valu_roofline(f"models:{name}", kern_ms, n)
        if vr["frac"] is not None:
            # VALU-bound models: the fraction of the chip's VALU issue slots, from committed counters of this kernel
            per[name]["valu_roofline"] = vr
        total_t += elapsed / reps
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        with tempfile.TemporaryDirectory() as tmp:
            merl_path = None
            if "Merl" in names:
                merl_path = os.path.join(tmp, "synthetic.binary")
                ld, lo = fit.merl_linearizer().directions()
                merl.write_binary(merl_path, merl.encode(bbm_amd.CookTorrance().eval(ld, lo).cpu().numpy()))
            cpu = cpu_models(names, sets[0][0], sets[0][1], args.cpu_seconds, merl_path)
    if rank == 0:
        _line(args, world, "BSDF evals/s (eval), all single bsdfmodels, 10M shared pairs per GPU (config 3)",
              len(names) * n * world * args.steps / total_t, "pairs/s", total_t / len(names),
              {"workload": f"{len(names)} models x eval over {n} pairs per GPU, one kernel per model (replayed as a "
                           f"graph of {reps} launches per step over {MODEL_SETS} distinct input/output sets, "
                           f"{MODEL_SETS * 36 * n / 1e9:.2f} GB > the 256 MiB Infinity Cache)",
               "pairs_per_gpu": n, "operand_sets": MODEL_SETS, "parallelism": f"dp{world} (independent shards)"},
              dict({"scaling": "weak", "per_model": per}, **({"cpu_baseline": cpu} if cpu else {})))


# models of config 4 whose sampler has an exact-mode twin (math.hpp exact_sample_t: Beckmann's glibc erff / logf,
# GGX's glibc sinf / cosf)
EXACT_SAMPLERS = ("CookTorrance", "GGX")


def bench_sample(args, dist, rank, world):
    per_gpu = 125_000_000
    slots = 8
    lib = _lib.load()
    outs = torch.from_numpy(check.reflectance_outs(slots)).cuda()
    stream = torch.cuda.current_stream()
    res = {}
    total_t = 0.0
    elapsed_of = {}
    for name in _subset(args, ("CookTorrance", "GGX")):
        m = bbm_amd.BsdfModel(name)
        d = check.CheckDesc()
        d.test, d.nslots, d.seed, d.begin, d.n = check.REFLECTANCE, slots, SEED, rank * (per_gpu // slots), per_gpu // slots
        d.slot_x, d.slot_y, d.slot_z = outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr()
        d.importance = 1
        acc = torch.empty((slots, check.ACC), dtype=torch.float64, device="cuda")
        wsb = int(lib.bbm_hip_check_workspace_size(ctypes.byref(d)))
        ws = torch.empty(max(wsb // 8, 1), dtype=torch.float64, device="cuda")

        def step():
            _lib.check(lib.bbm_hip_check(m.model_id, m._pptr(), m._params.size, ctypes.byref(d), acc.data_ptr(), None,
                                         ws.data_ptr(), wsb, _stream_ptr(stream)))

        elapsed, kern_ms = _timed(step, args, dist, stream)
        a = check._gather_acc(acc.cpu().numpy(), dist)
        exact_ms = None
        if world == 1 and not args.no_exact and name in EXACT_SAMPLERS:
            # the same steps on the sampler's exact-mode twin (glibc erff / logf in the Beckmann sampler)
            prev = bbm_amd.set_exact_subnormals(True)
            try:
                exact_ms = _timed(step, args, dist, stream)[1]
            finally:
                bbm_amd.set_exact_subnormals(prev)
        total = (per_gpu // slots) * slots * world
        est = a[:, :3] / float(total // slots)
        refl = m.reflectance(outs).cpu().numpy().T
        res[name] = {"samples_per_s": total * args.steps / elapsed, "kernel_ms": kern_ms,
                     "samples_per_dispatch": (per_gpu // slots) * slots,
                     "exact_mode_kernel_ms": exact_ms,
                     "roofline": valu_roofline(f"sample:{name}", kern_ms, (per_gpu // slots) * slots),
                     "estimate_vs_reflectance": [[float(x) for x in est[k]] + [float(y) for y in refl[k]] for k in (0, slots - 1)]}
        total_t += elapsed
        elapsed_of[name] = elapsed
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_sample(list(res), outs, slots, args.cpu_seconds)
    if rank == 0:
        # the workload value is the first model's own rate (CookTorrance, the headline model), not an average over
        # the models timed; every model's figure is in per_model
        head = next(iter(res))
        _line(args, world, f"importance-sample->eval->pdf samples/s, microfacet {head}, 125M samples per GPU "
              "(config 4)", res[head]["samples_per_s"], "samples/s", elapsed_of[head],
              {"workload": f"checkBsdf reflectance test, importance sampling, {slots} theta_out x "
                           f"{per_gpu // slots} samples per GPU, in-kernel reduction",
               "samples_per_gpu": per_gpu, "parallelism": f"dp{world} (sample shards, one gather at the end)"},
              dict({"scaling": "weak", "per_model": res, "roofline": res[head]["roofline"]},
                   **({"cpu_baseline": cpu} if cpu else {})))


def _merl_from(source):
    """A Merl model read from a MERL-format .binary that holds `source` evaluated at the MERL bin centres."""
    din, dout = fit.merl_linearizer().directions()
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "synthetic.binary")
        merl.write_binary(path, merl.encode(source.eval(din, dout).cpu().numpy()))
        return bbm_amd.Merl(path)


FIT_MATERIAL = ("bagher_sgd.fit", "alum-bronze")     # fits/bagher_sgd.fit:3, SURVEY §8(d) C5
# the material's line of the published fit file, verbatim (data: the fitted parameter values; the GPU box has no
# /root/reference to read it from)
FIT_LINE = ("alum-bronze = Aggregate(Lambertian(albedo = [0.0478786, 0.0313514, 0.0200638]), Bagher(albedo = [0.0"
            "364976, 0.664975, 0.268836], alpha = [0.014832, 0.0300126, 0.0490339], p = [0.459076, 0.450056, 0.52"
            "9272], eta = [[6.05524, 0.235756, 0.580647], [5.05524, 0.182842, 0.476088]], K = [46.3841, 24.5961, "
            "14.8261], Lambda = [2.60672, 2.97371, 2.7827], c = [1.12717e-07, 1.06401e-07, 5.27952e-08], k = [47."
            "783, 36.2767, 31.6066], theta0 = [0.205635, 0.066289, -0.0661091]))")


def fit_material():
    """(name, model) of the config-5 material: FIT_LINE ("name = model string", fits/*.fit's format) split at
    " = " and the model built by the library's own C-ABI parser (bbm_amd.parse_model -> bbm_hip_parse_model_tree,
    the runtime fromString an FFI caller of the fits/ files would use)."""
    name, mstr = FIT_LINE.split(" = ", 1)
    assert name == FIT_MATERIAL[1]
    return name, bbm_amd.parse_model(mstr)


def bench_fit(args, dist, rank, world):
    """Config 5.  The measured reference is the published fit fits/bagher_sgd.fit:3 (alum-bronze) written at the
    MERL bin centres into a MERL-format .binary and read back through bbm_amd.Merl, as a real MERL file would be;
    the fitted model is Aggregate(Lambertian, Bagher) at its defaults.  value: probe-pair evaluations/s of a
    compass step's 2P probes (one bbm_hip_loss launch + the RCCL all-reduce), K timed steps; then the compass
    search runs from the defaults to convergence (compass.h:82-140, step size < eps) or --fit-max-steps /
    --fit-max-seconds, and the
    line reports its steps, wall time per step and the loss before / after."""
    name = "Aggregate<Lambertian,Bagher>"
    mat, material = fit_material()
    fitted = bbm_amd.BsdfModel(name)
    lin = fit.merl_linearizer()
    reference = _merl_from(material)
    loss = fit.SampledLoss(fitted, reference, "standardLog", lin, dist=dist)
    idx = fitted.parameter_indices(fit.ALL)
    probes = np.repeat(fitted.parameter_values()[None], 2 * len(idx), axis=0)
    for k, j in enumerate(idx):
        probes[2 * k, j] *= np.float32(1.01)
        probes[2 * k + 1, j] *= np.float32(0.99)
    stream = torch.cuda.current_stream()
    elapsed, kern_ms = _timed(lambda: loss.probe_sums(probes), args, dist, stream)
    # the fit itself, from the defaults
    comp = fit.Compass(loss)
    loss0 = float(comp.loss_value)
    t0 = time.perf_counter()
    steps = 0
    while not comp.is_converged() and steps < args.fit_max_steps and time.perf_counter() - t0 < args.fit_max_seconds:
        comp.step()
        steps += 1
    torch.cuda.synchronize()
    fit_s = time.perf_counter() - t0
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_fit(name, fitted, material, lin, args.cpu_seconds)
    if rank == 0:
        pairs = lin.size()
        _line(args, world, "fitting-loss probe-pair evals/s, Aggregate(Lambertian, Bagher), MERL grid, 2P probes per "
              "compass step (config 5)", len(probes) * pairs * args.steps / elapsed, "probe-pairs/s", elapsed,
              {"workload": f"{len(probes)} probes x {pairs} MERL pairs per compass step (standardLog), sharded grid; "
                           f"reference = Merl model read from a MERL .binary holding fits/{FIT_MATERIAL[0]} "
                           f"'{mat}' (line 3) at the MERL bin centres",
               "material": f"fits/{FIT_MATERIAL[0]}:3 {mat}",
               "probes": len(probes), "pairs": pairs, "parallelism": f"dp{world} (grid shards, all-reduce of "
                                                                      f"{len(probes)} doubles per step)"},
              {"scaling": "strong", "compass_steps_per_s": args.steps / elapsed, "kernel_ms": kern_ms,
               "probe_pairs_per_dispatch": len(probes) * (pairs // world),
               "roofline": valu_roofline("fit:Aggregate", kern_ms, len(probes) * (pairs // world)),
               "fit": {"from": "Aggregate<Lambertian,Bagher> defaults", "steps": steps,
                       "converged": comp.is_converged(), "max_steps": args.fit_max_steps,
                       "max_seconds": args.fit_max_seconds, "seconds": fit_s,
                       "ms_per_compass_step": fit_s * 1e3 / max(steps, 1), "loss_start": loss0,
                       "loss_end": float(comp.loss_value), "final_step_size": float(comp.step_size)},
               **({"cpu_baseline": cpu} if cpu else {})})


def bench_f64(args, dist, rank, world):
    """doubleRGB (bbm_hip_eval_pdf_f64): --model's eval+pdf over --pairs f64 pairs per GPU (HIP-event timed, HBM
    roofline at 80 B/pair: 48 B in + 32 B out), and every doubleRGB model over 10M shared pairs (graph-timed)."""
    begin, n = bh.shard(args.pairs, rank, world, args.scaling)
    din = bbm_amd.fill_directions(SEED, 0, begin, n, mode=0).double()
    dout = bbm_amd.fill_directions(SEED, 1, begin, n, mode=0).double()
    rgb = torch.empty((3, n), dtype=torch.float64, device="cuda")
    pdf = torch.empty((n,), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()
    model = bbm_amd.BsdfModel(args.model)
    elapsed, kern_ms = _timed(lambda: model.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=stream), args, dist, stream)
    ok = bool(torch.isfinite(pdf).all()) and float(rgb[0].abs().max()) > 0
    bpp = 80
    gbs = bpp * n / (kern_ms * 1e-3) / 1e9
    del din, dout, rgb, pdf
    m10 = 10_000_000
    din = bbm_amd.fill_directions(SEED, 0, rank * m10, m10, mode=0).double()
    dout = bbm_amd.fill_directions(SEED, 1, rank * m10, m10, mode=0).double()
    rgb = torch.empty((3, m10), dtype=torch.float64, device="cuda")
    pdf = torch.empty((m10,), dtype=torch.float64, device="cuda")
    per = {}
    lib = _lib.load()
    for name in _subset(args, [m for i, m in enumerate(bbm_amd.model_names()) if lib.bbm_hip_model_has_f64(i) == 1]):
        mm = bbm_amd.BsdfModel(name)
        graph = _graph(lambda s: mm.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=s), GRAPH_REPS)
        _, step_ms = _timed(graph.replay, args, dist, stream)
        k = step_ms / GRAPH_REPS
        b = 48 if name in Z_ONLY else bpp    # Lambertian reads only z: 16 B in + 32 B out
        per[name] = {"kernel_ms": k, "pairs_per_s": m10 / (k * 1e-3), "GB_s": b * m10 / (k * 1e-3) / 1e9,
                     "roofline_frac": b * m10 / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, "bytes_per_pair": b}
    if rank == 0:
        global_pairs = n * world if args.scaling == "weak" else args.pairs
        d = {"metric": f"BSDF evals/s (eval+pdf), {args.model}, doubleRGB (f64)", "value": global_pairs * args.steps / elapsed,
             "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
             "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": args.scaling,
             "vs_baseline": None, "dtype": "f64", "data": "synthetic (counter-based directions, widened to f64 on device)",
             "config": {"workload": f"{args.model} fused eval+pdf, {n} pairs per GPU, f64 SoA (doubleRGB)",
                        "pairs_per_gpu": n, "parallelism": f"dp{world} (independent shards, no collective)"},
             "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": gbs / HBM_PEAK_GBS, "traffic": None, "kernel": f"k_eval_pdf_f64<{args.model}>",
                          "kernel_ms": kern_ms, "bytes_per_pair": bpp},
             "outputs_ok": ok, "per_model_10M": per}
        print(json.dumps(d), flush=True)


def run(args, dist, rank, world):
    {"models": bench_models, "sample": bench_sample, "fit": bench_fit, "f64": bench_f64}[args.workload](
        args, dist, rank, world)
