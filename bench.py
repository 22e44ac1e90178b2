#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: CookTorrance eval+pdf pairs/s, 100M pairs per GPU, f32.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P] [--model NAME] [--no-cpu]

One step = one fused eval+pdf pass (bbm_hip_eval_pdf) of the model over the GPU's shard of
synthetic direction pairs already resident in HBM (SoA f32, generated on the device by the
counter-based bbm_hip_fill_directions before timing; upper hemisphere, every lane active).
Multi-GPU (torchrun, one process per GPU): every rank owns a contiguous shard of the global batch
(weak scaling: P pairs per GPU), no data-path collective; barrier + synchronize bracket the K
timed steps and the slowest rank's time is used.  value = all pairs processed / that time.

roofline: the dominant (only) kernel, k_eval_pdf_v4<CookTorrance>, timed with HIP events on the
stream it is launched on; algorithmic bytes = 40 B/pair (6 x 4 B in + 3 x 4 B RGB + 4 B pdf,
SURVEY.md §8d); peak = 8 TB/s HBM3E (MI355X_MICROARCH.md).  traffic: PMC-measured HBM bytes per
launch from profiles/ (see DESIGN.md §5), or null.

cpu_baseline (rank 0, N=1 only): the reference itself (oracle/_ref/libbbm_ref.so: the reference
headers compiled with the native floatRGB backbone, OpenMP over the host cores we were given) on a
bounded sample of the same pairs (copied back from the GPU), repeated for ~10 s.
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

BYTES_PER_PAIR = 40           # 24 B in + 16 B out (eval RGB + pdf), f32 SoA
# models whose eval+pdf never reads in.xy / out.xy: only z is loaded (8 B in + 16 B out)
BYTES_PER_PAIR_MODEL = {"Lambertian": 24}
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec
SEED = 0xBB5EED
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="after the W warmup steps, keep stepping (untimed) until this much wall time has passed "
                         "since warmup began: MI355X clocks take ~50 back-to-back launches to settle after a load change")
    ap.add_argument("--pairs", type=int, default=100_000_000, help="pairs per GPU")
    ap.add_argument("--model", default="CookTorrance")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--workload", default="evalpdf", choices=["evalpdf", "models", "sample", "fit"],
                    help="evalpdf: the BASELINE metric (config 2, default); models: every model's eval over shared "
                         "pairs (config 3); sample: importance-sample -> eval -> pdf MC loop (config 4); fit: "
                         "multi-probe fitting loss of a compass step over the MERL grid (config 5)")
    return ap.parse_args()


def cpu_baseline(model, din, dout, seconds):
    """Reference (or, if the prebuilt shim is absent, the C restatement) on a bounded sample."""
    from tests import oracle_util as ou
    n = min(din.shape[1], 8_000_000)
    hin = np.ascontiguousarray(din[:, :n].cpu().numpy())
    hout = np.ascontiguousarray(dout[:, :n].cpu().numpy())
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    params = model.parameter_values()
    if ou.ref() is not None:
        kind, fn = "reference", ou.ref_eval_pdf
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
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": done / el, "unit": "pairs/s", "cores": threads, "kind": kind,
            "sample": f"{n} pairs of the same synthetic batch, {done // n} passes in {el:.1f} s, "
                      f"{model.name} eval+pdf via {'oracle/_ref (reference headers, native floatRGB)' if kind == 'reference' else 'oracle/port'}, "
                      f"OpenMP {threads} threads on {cpu_model}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(0)

    import bbm_amd
    if args.workload != "evalpdf":
        from tools import bench_configs
        bench_configs.run(args, dist, rank, world)
        if dist:
            dist.destroy_process_group()
        return
    model = bbm_amd.BsdfModel(args.model)
    n = args.pairs
    dev = torch.device("cuda", torch.cuda.current_device())
    from bbm_amd.shard import weak_range
    # this rank's shard [rank*n, (rank+1)*n) of the global batch, regenerated on device
    begin, _ = weak_range(n, rank)
    din = bbm_amd.fill_directions(SEED, 0, begin, n, mode=0)
    dout = bbm_amd.fill_directions(SEED, 1, begin, n, mode=0)
    rgb = torch.empty((3, n), dtype=torch.float32, device=dev)
    pdf = torch.empty((n,), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()

    tw = time.perf_counter()
    for _ in range(args.warmup):
        model.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=stream)
    torch.cuda.synchronize()
    settle_steps = 0
    while time.perf_counter() - tw < args.settle_s:
        for _ in range(10):
            model.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=stream)
        settle_steps += 10
        torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        model.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=stream)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    # sanity: outputs finite and non-trivial
    ok = bool(torch.isfinite(pdf).all()) and float(rgb[0].abs().max()) > 0

    if rank == 0:
        total_pairs = n * world * args.steps
        bpp = BYTES_PER_PAIR_MODEL.get(args.model, BYTES_PER_PAIR)
        achieved = bpp * n / (kern_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(TRAFFIC_FILE):
            try:
                with open(TRAFFIC_FILE) as f:
                    tr = json.load(f)
                if tr.get("model") == args.model and tr.get("pairs") == n:
                    traffic = tr.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        line = {
            "metric": "BSDF evals/s (eval+pdf) per GPU, CookTorrance 100M pairs; 1/2/4/8-GPU scaling"
            if args.model == "CookTorrance" else f"BSDF evals/s (eval+pdf), {args.model}",
            "value": total_pairs / elapsed,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-based directions on the upper hemisphere, generated on device)",
            "config": {"workload": f"{args.model} fused eval+pdf, {n} pairs per GPU, f32 SoA",
                       "model": str(model), "pairs_per_gpu": n, "global_pairs": n * world,
                       "parallelism": f"dp{world} (independent shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": f"k_eval_pdf_v4<{args.model}>", "kernel_ms": kern_ms,
                         "bytes_per_pair": bpp},
            "outputs_ok": ok,
            "settle": {"seconds": args.settle_s, "extra_untimed_steps": settle_steps},
        }
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(model, din, dout, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
