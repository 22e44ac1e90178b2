#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: CookTorrance eval+pdf pairs/s, 100M pairs per GPU, f32.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong] [--pairs P] [--model NAME]
                    [--no-cpu] [--workload evalpdf|models|sample|fit|f64|lambertian-cpu|selftest]

One step = one fused eval+pdf pass (bbm_hip_eval_pdf) of the model over the GPU's shard of synthetic
direction pairs already resident in HBM (SoA f32, generated on the device by the counter-based
bbm_hip_fill_directions before timing; upper hemisphere, every lane active).

Multi-GPU: one process per GPU.  Under torchrun the launcher's WORLD_SIZE is used (and must equal --gpus);
`python bench.py --gpus N` without a launcher starts torchrun itself as a child process before anything
touches the GPU.  Every rank owns a contiguous shard of the global batch and regenerates it from
(seed, global index): no data-path collective.  --scaling weak (default): P pairs per GPU, the global batch
grows with N; --scaling strong: P pairs in total, split over the N ranks.  Barrier + synchronize bracket the
K timed steps; the slowest rank's time is the job's time; value = all pairs processed / that time.  The line
carries every rank's time and the rank count the process group saw.

roofline: the dominant (only) kernel, k_eval_pdf_v4<CookTorrance>, timed with HIP events on the stream it
is launched on; algorithmic bytes = 40 B/pair (6 x 4 B in + 3 x 4 B RGB + 4 B pdf);
peak = 8 TB/s HBM3E (MI355X_MICROARCH.md).  traffic: PMC-measured HBM bytes per launch from profiles/
(see DESIGN.md §5), or null.

cpu_baseline (rank 0, N=1 only): the reference itself (oracle/_ref/libbbm_ref.so: the reference headers
compiled with the native floatRGB backbone, OpenMP over every host thread this process may run on) on a
bounded sample of the same pairs (copied back from the GPU), repeated for ~10 s.

--workload selftest: the launcher / rendezvous / timing harness alone on the CPU (gloo, a trivial step);
no GPU and no BSDF work -- it exists so the multi-rank path can be tested without a GPU.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tools import bench_harness as bh  # noqa: E402

BYTES_PER_PAIR = 40           # 24 B in + 16 B out (eval RGB + pdf), f32 SoA
# models whose eval+pdf never reads in.xy / out.xy: only z is loaded (8 B in + 16 B out)
BYTES_PER_PAIR_MODEL = {"Lambertian": 24}
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec
SEED = 0xBB5EED
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")
METRIC = "BSDF evals/s (eval+pdf) per GPU, CookTorrance 100M pairs; 1/2/4/8-GPU scaling"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default: WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="after the W warmup steps, keep stepping (untimed) until this much wall time has passed "
                         "since warmup began: MI355X clocks take ~50 back-to-back launches to settle after a load change")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --pairs per GPU; strong: --pairs in total, split over the ranks")
    ap.add_argument("--pairs", type=int, default=100_000_000, help="pairs per GPU (weak) or in total (strong)")
    ap.add_argument("--model", default="CookTorrance")
    ap.add_argument("--models", default=None, help="comma-separated subset of models for --workload models|sample "
                                                   "(counter passes profile one model at a time)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-exact", action="store_true", help="evalpdf, sample: skip the exact mode's timing")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="evalpdf: time the K steps as HIP-graph replays of R launches (K/R replays, R | K) instead of "
                         "one Python-side launch per step; auto = when this rank's shard is below --graph-below pairs "
                         "(a ~0.2 ms kernel, e.g. 12.5M pairs per GPU under --scaling strong on 8 GPUs). Both figures "
                         "are reported; value is the graph-timed one when the graph is used")
    ap.add_argument("--graph-below", type=int, default=30_000_000)
    ap.add_argument("--fit-max-steps", type=int, default=200000, help="fit: compass steps cap for the convergence run")
    ap.add_argument("--fit-max-seconds", type=float, default=120.0, help="fit: wall-time cap for the convergence run")
    ap.add_argument("--workload", default="evalpdf",
                    choices=["evalpdf", "models", "sample", "fit", "f64", "lambertian-cpu", "selftest"],
                    help="evalpdf: the BASELINE metric (config 2, default); models: every model's eval over shared "
                         "pairs (config 3); sample: importance-sample -> eval -> pdf MC loop (config 4); fit: "
                         "multi-probe fitting loss of a compass step over the MERL grid (config 5); f64: the doubleRGB "
                         "path (--model over --pairs f64 pairs + every doubleRGB model); lambertian-cpu: config 1, the "
                         "native CPU backbone's Lambertian eval over 1M pairs (no GPU); selftest: the "
                         "multi-rank harness on the CPU (gloo), no GPU")
    return ap.parse_args(argv)


def cpu_baseline(model, din, dout, seconds):
    """Reference (or, if the prebuilt shim is absent, the C restatement) on a bounded sample, on every host
    thread this process may run on."""
    from tests import oracle_util as ou
    n = min(din.shape[1], 8_000_000)
    hin = np.ascontiguousarray(din[:, :n].cpu().numpy())
    hout = np.ascontiguousarray(dout[:, :n].cpu().numpy())
    aff, phys, smt, quota, cpu_model = bh.cpu_topology()
    # every CPU this process may use: the affinity mask, capped by the cgroup's CPU quota when there is one (the
    # GPU box grants 16 CPUs of a 256-thread host: 256 OpenMP threads under that quota were throttled to 1/6 of
    # the 16-thread rate, profiles/r02_bench_cpu256.json)
    threads = aff if quota is None else max(1, min(aff, int(-(-quota // 1))))
    params = model.parameter_values()
    if ou.ref() is not None:
        kind = "reference"
        fn = lambda *a, **k: ou._evalpdf(ou.ref_bench().bbmref_eval_pdf, *a[:4], 3, 0, k["nthreads"])   # noqa: E731
    else:
        kind, fn = "port", ou.port_eval_pdf
    fn(model.name, params, hin[:, :100_000], hout[:, :100_000], nthreads=threads)   # warm-up
    done, t0 = 0, time.perf_counter()
    while True:
        fn(model.name, params, hin, hout, nthreads=threads)
        done += n
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el, "unit": "pairs/s", "cores": threads, "kind": kind,
            "affinity_threads": aff, "physical_cores": phys, "smt_threads_per_core": smt, "cgroup_cpu_quota": quota,
            "sample": f"{n} pairs of the same synthetic batch, {done // n} passes in {el:.1f} s, "
                      f"{model.name} eval+pdf via {'oracle/_ref (reference headers, native floatRGB, -O3 Release build)' if kind == 'reference' else 'oracle/port'}, "
                      f"OpenMP {threads} threads = every CPU this process may use (affinity mask: {aff} threads on "
                      f"{phys} physical cores x {smt} SMT{'' if quota is None else f'; cgroup CPU quota {quota:g} CPUs'}) "
                      f"on {cpu_model}"}


def lambertian_cpu(args):
    """Config 1 (BASELINE.json configs[0]): Lambertian eval on the native CPU backbone, 1M (in, out) pairs -- plumbing,
    no GPU.  The reference itself (oracle/_ref: the reference headers with the native floatRGB backbone; oracle/port, the
    C restatement, where the prebuilt shim is absent) evaluates the same counter-generated pairs the GPU path would
    (tests/oracle_util.dirgen_numpy restates bbm_hip_fill_directions), K timed passes after W untimed ones, OpenMP over
    every CPU this process may use; the single-thread rate beside it."""
    from tests import oracle_util as ou
    from tools.bench_configs import cpu_threads, _ref_eval_call
    n = 1_000_000
    din = np.ascontiguousarray(ou.dirgen_numpy(SEED, 0, 0, n, mode=0))
    dout = np.ascontiguousarray(ou.dirgen_numpy(SEED, 1, 0, n, mode=0))
    params = np.array([0.5, 0.5, 0.5], np.float32)      # Lambertian's default albedo (lambertian.h:27)
    lib, kind = ou.ref_bench(), "reference"
    if lib is None:
        lib, kind = ou.port(), "port"
        fn = lib.bbmport_eval_pdf
        import types
        lib = types.SimpleNamespace(bbmref_eval_pdf=fn)
    threads, tdesc = cpu_threads()
    res = {}
    for t in (threads, 1):
        call = _ref_eval_call(lib, "Lambertian", params, din, dout, 1, t)
        steps = args.steps if t == threads else max(3, args.steps // 20)
        for _ in range(args.warmup if t == threads else 1):
            call()
        t0 = time.perf_counter()
        for _ in range(steps):
            call()
        res[t] = (steps, time.perf_counter() - t0)
    steps, el = res[threads]
    print(json.dumps({"metric": "Lambertian evals/s, native CPU backbone, 1M (in, out) pairs (config 1)",
                      "value": n * steps / el, "unit": "pairs/s", "n_gpus": 0, "steps": steps, "warmup": args.warmup,
                      "ms_per_step": el * 1e3 / steps, "higher_is_better": True, "scaling": "none",
                      "vs_baseline": None, "dtype": "f32",
                      "data": "synthetic (the counter-based directions of bbm_hip_fill_directions, restated in numpy)",
                      "config": {"workload": f"Lambertian eval (no pdf) over {n} pairs on the host CPU, {kind} "
                                             f"(oracle/_ref = the reference headers, native floatRGB backbone)",
                                 "pairs": n, "parallelism": f"OpenMP {threads} threads"},
                      "cores": threads, "cpu": tdesc, "kind": kind,
                      "single_thread": {"value": n * res[1][0] / res[1][1], "steps": res[1][0]}}), flush=True)


def selftest(args, dist, rank, world):
    """Harness only: a trivial CPU step under the same launch / barrier / max-over-ranks timing, with the evalpdf
    workload's --graph choice (a 'graph' here is R steps issued by one call, R = bh.graph_reps(K))."""
    begin, n = bh.shard(args.pairs, rank, world, args.scaling)
    x = torch.arange(n, dtype=torch.float32)
    elapsed, _, per_rank, settle = bh.timed(lambda: x.sum(), args, dist, gpu=False)
    use_graph = args.graph == "on" or (args.graph == "auto" and n < args.graph_below)
    timing = {"launch_timed": {"elapsed_s": elapsed, "rank_ms_per_step": [t * 1e3 / args.steps for t in per_rank]}}
    if use_graph:
        reps = bh.graph_reps(args.steps)
        g_el, _, g_per, _ = bh.timed(lambda: [x.sum() for _ in range(reps)],
                                     argparse.Namespace(**{**vars(args), "steps": args.steps // reps}), dist, gpu=False)
        timing["graph_timed"] = {"elapsed_s": g_el, "launches_per_replay": reps, "replays": args.steps // reps,
                                 "rank_ms_per_step": [t * 1e3 / args.steps for t in g_per]}
        elapsed, per_rank = g_el, g_per
    if rank == 0:
        total = (n * world if args.scaling == "weak" else args.pairs) * args.steps
        print(json.dumps({"metric": "bench harness self-test (CPU, no BSDF work)", "value": total / elapsed,
                          "unit": "units/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
                          "scaling": args.scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "config": {"workload": "selftest", "units_per_rank": n,
                                     "parallelism": f"dp{world}"},
                          "ranks_seen": dist.get_world_size() if dist else 1,
                          "rank_ms_per_step": [t * 1e3 / args.steps for t in per_rank],
                          "timing": dict(timing, value_from="graph_timed" if use_graph else "launch_timed")}),
              flush=True)


def main(argv=None):
    args = parse(argv)
    if bh.needs_launch(args.gpus):
        # no GPU call has been made in this process: start the ranks as a child and exit with its status
        sys.exit(bh.launch(args.gpus, os.path.abspath(__file__), sys.argv[1:] if argv is None else argv))
    world, rank, local = bh.world_from_env(args.gpus)
    if args.workload == "lambertian-cpu":
        lambertian_cpu(args)
        return
    if args.workload == "selftest":
        dist = bh.init(world, local, "gloo")
        selftest(args, dist, rank, world)
        if dist:
            dist.destroy_process_group()
        return
    dist = bh.init(world, local, "nccl")
    if dist is None:
        torch.cuda.set_device(0)

    import bbm_amd
    if args.workload != "evalpdf":
        from tools import bench_configs
        bench_configs.run(args, dist, rank, world)
        if dist:
            dist.destroy_process_group()
        return
    model = bbm_amd.BsdfModel(args.model)
    begin, n = bh.shard(args.pairs, rank, world, args.scaling)
    dev = torch.device("cuda", torch.cuda.current_device())
    # this rank's contiguous shard [begin, begin + n) of the global batch, regenerated on device
    din = bbm_amd.fill_directions(SEED, 0, begin, n, mode=0)
    dout = bbm_amd.fill_directions(SEED, 1, begin, n, mode=0)
    rgb = torch.empty((3, n), dtype=torch.float32, device=dev)
    pdf = torch.empty((n,), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()

    launch = lambda s=stream: model.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=s)   # noqa: E731
    elapsed, kern_ms, per_rank, settle = bh.timed(launch, args, dist, stream)
    use_graph = args.graph == "on" or (args.graph == "auto" and n < args.graph_below)
    timing = {"launch_timed": {"elapsed_s": elapsed, "kernel_ms": kern_ms, "rank_ms_per_step":
                               [t * 1e3 / args.steps for t in per_rank]}}
    if use_graph:
        # the same K steps as R-launch graph replays: the host issues one replay per R steps
        reps = bh.graph_reps(args.steps)
        graph = bh.capture(launch, reps)
        g_el, g_ms, g_per, _ = bh.timed(graph.replay, argparse.Namespace(**{**vars(args), "steps": args.steps // reps,
                                                                             "warmup": 2, "settle_s": 0.1}), dist, stream)
        timing["graph_timed"] = {"elapsed_s": g_el, "kernel_ms": g_ms / reps, "launches_per_replay": reps,
                                 "replays": args.steps // reps,
                                 "rank_ms_per_step": [t * 1e3 / args.steps for t in g_per]}
        elapsed, kern_ms, per_rank = g_el, g_ms / reps, g_per

    # the same K steps in the exact-subnormal mode (bbm_hip_set_exact_subnormals: every lane the reference's float;
    # the Beckmann microfacet models only), reported beside the default mode's figure, not as the value
    exact = None
    if world == 1 and not args.no_exact:
        prev = bbm_amd.set_exact_subnormals(True)
        try:
            e_el, e_ms, _, _ = bh.timed(launch, argparse.Namespace(**{**vars(args), "warmup": 5, "settle_s": 0.1}),
                                        dist, stream)
        finally:
            bbm_amd.set_exact_subnormals(prev)
        exact = {"value": n * args.steps / e_el, "kernel_ms": e_ms,
                 "roofline_frac": BYTES_PER_PAIR_MODEL.get(args.model, BYTES_PER_PAIR) * n / (e_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                 "note": "bit-identical to the reference on every lane (tests/test_gpu_parity.py::"
                         "test_exact_subnormal_mode_is_bit_exact); default mode: outputs below ~1e-30 may differ in the last bit"}

    # sanity: outputs finite and non-trivial
    ok = bool(torch.isfinite(pdf).all()) and float(rgb[0].abs().max()) > 0

    if rank == 0:
        global_pairs = n * world if args.scaling == "weak" else args.pairs
        total_pairs = global_pairs * args.steps
        bpp = BYTES_PER_PAIR_MODEL.get(args.model, BYTES_PER_PAIR)
        achieved = bpp * n / (kern_ms * 1e-3) / 1e9
        traffic = None
        for tf in (os.path.join(ROOT, "profiles", f"traffic_{args.model}.json"), TRAFFIC_FILE):
            try:
                with open(tf) as f:
                    tr = json.load(f)
            except (OSError, ValueError):
                continue
            if tr.get("model") == args.model and tr.get("pairs") == n:
                traffic = tr.get("hbm_bytes_per_launch")
                break
        line = {
            "metric": METRIC if args.model == "CookTorrance" else f"BSDF evals/s (eval+pdf), {args.model}",
            "value": total_pairs / elapsed,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-based directions on the upper hemisphere, generated on device)",
            "config": {"workload": f"{args.model} fused eval+pdf, {n} pairs per GPU, f32 SoA",
                       "model": str(model), "pairs_per_gpu": n, "global_pairs": global_pairs,
                       "parallelism": f"dp{world} (independent shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": f"k_eval_pdf_v4<{args.model}>", "kernel_ms": kern_ms,
                         "bytes_per_pair": bpp},
            "ranks_seen": dist.get_world_size() if dist else 1,
            "rank_ms_per_step": [t * 1e3 / args.steps for t in per_rank],
            "timing": dict(timing, value_from="graph_timed" if use_graph else "launch_timed"),
            "outputs_ok": ok,
            "settle": {"seconds": args.settle_s, "extra_untimed_steps": settle},
        }
        if exact is not None:
            line["exact_subnormals_mode"] = exact
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(model, din, dout, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
