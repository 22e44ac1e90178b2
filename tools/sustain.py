#!/usr/bin/env python3
"""Sustained-load behaviour of the eval+pdf kernel vs the trivial-compute roofline probe.

    python tools/sustain.py [--pairs 100000000] [--launches 200] [--models CookTorrance,GGX]

Launches each kernel back to back, times every launch with HIP events on its stream and prints
percentiles plus the per-launch series (to see clock/power transients).  Writes
gpurun_out/sustain.json.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def series(launch, s, k):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for i in range(k):
        ev[i][0].record(s)
        launch()
        ev[i][1].record(s)
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) for a, b in ev])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100_000_000)
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--models", default="CookTorrance")
    args = ap.parse_args()
    import bbm_amd
    n = args.pairs
    s = torch.cuda.current_stream()
    din = bbm_amd.fill_directions(0xBB5EED, 0, 0, n, mode=0)
    dout = bbm_amd.fill_directions(0xBB5EED, 1, 0, n, mode=0)
    rgb = torch.empty((3, n), dtype=torch.float32, device="cuda")
    pdf = torch.empty((n,), dtype=torch.float32, device="cuda")
    res = {}
    probe = os.path.join(ROOT, "tools", "libroofprobe.so")
    runs = []
    if os.path.exists(probe):
        lib = ctypes.CDLL(probe)
        lib.roofprobe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                  ctypes.c_void_p]
        in_ptrs = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in (din[0], din[1], din[2], dout[0], dout[1], dout[2])])
        out_ptrs = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in (rgb[0], rgb[1], rgb[2], pdf)])
        blocks = (n // 4 + 255) // 256
        runs.append(("probe_nt", lambda: lib.roofprobe(1, in_ptrs, out_ptrs, n, blocks, s.cuda_stream)))
    for name in args.models.split(","):
        m = bbm_amd.BsdfModel(name)
        runs.append((name, lambda m=m: m.eval_pdf(din, dout, rgb=rgb, pdf=pdf, stream=s)))
    for name, fn in runs:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = series(fn, s, args.launches)
        gbs = 40 * n / (t * 1e-3) / 1e9
        res[name] = {"ms": t.tolist(), "p10": float(np.percentile(t, 10)), "p50": float(np.median(t)),
                     "p90": float(np.percentile(t, 90)), "mean": float(t.mean()),
                     "GBps_mean": float(40 * n / (t.mean() * 1e-3) / 1e9)}
        print(f"{name:16s} mean {t.mean():.3f} ms  p10 {res[name]['p10']:.3f}  p50 {res[name]['p50']:.3f}  "
              f"p90 {res[name]['p90']:.3f}  -> {res[name]['GBps_mean']:.0f} GB/s (40 B/pair)", flush=True)
        print("   series:", " ".join(f"{x:.3f}" for x in t[:: max(1, len(t) // 40)]), flush=True)
        # idle gap, so every kernel starts from the same thermal/power state
        torch.cuda._sleep(int(2e9))
        torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sustain.json"), "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
