#!/usr/bin/env python3
"""Calibrate the HBM ceiling of the eval+pdf access pattern on the GPU (tools/roofprobe.hip).

    python tools/roofprobe.py [--pairs 100000000]

Prints one line per (variant, grid) with GB/s computed from the algorithmic bytes.  Build the probe library with
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -o tools/libroofprobe.so tools/roofprobe.hip
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BYTES = {0: 40, 1: 40, 2: 40, 3: 24, 4: 16, 5: 8, 6: 40, 7: 24, 8: 16, 9: 40, 10: 40, 11: 40, 12: 40, 13: 40, 14: 40, 15: 40, 16: 40}
NAMES = {0: "plain 6in/4out", 1: "nontemporal 6in/4out", 2: "8 pairs/thread 6in/4out", 3: "read-only 6in",
         4: "write-only 4out", 5: "copy nt 1in/1out", 6: "nt 2 quads/lane 6in/4out", 7: "read-only nt 6in",
         8: "write-only nt 4out", 9: "nt chunk 16 tiles/WG", 10: "nt chunk 64 tiles/WG", 11: "nt chunk 4 tiles/WG",
         12: "AoS pair/lane", 13: "AoS 4 pairs/lane", 14: "AoS 4 pairs wave-strided",
         15: "nt loads, plain stores", 16: "plain loads, nt stores"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100_000_000)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import bbm_amd
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libroofprobe.so"))
    lib.roofprobe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                              ctypes.c_void_p]
    n = args.pairs
    ins = [bbm_amd.fill_directions(1, k, 0, n, mode=1) for k in range(2)]
    in_rows = [ins[0][0], ins[0][1], ins[0][2], ins[1][0], ins[1][1], ins[1][2]]
    outs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(4)]
    in_ptrs = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in in_rows])
    out_ptrs = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in outs])
    # the pair-array layout (variants 12-14): one 24 B-per-pair input array, one float4-per-pair output array
    aos_in = torch.stack(in_rows, dim=1).contiguous()
    aos_out = torch.empty(n, 4, dtype=torch.float32, device="cuda")
    aos_in_ptrs = (ctypes.c_void_p * 6)(*([aos_in.data_ptr()] * 6))
    aos_out_ptrs = (ctypes.c_void_p * 4)(*([aos_out.data_ptr()] * 4))
    s = torch.cuda.current_stream()
    res = []
    for v in [int(x) for x in os.environ.get("PROBE_VARIANTS", "0,1,2,3,4,5,6,7,8").split(",")]:
        for blocks in (1024, 2048, 4096, 8192, 16384, (n // 4 + 255) // 256):
            for _ in range(2):
                ip, op = (aos_in_ptrs, aos_out_ptrs) if 12 <= v <= 14 else (in_ptrs, out_ptrs)
                assert lib.roofprobe(v, ip, op, n, blocks, s.cuda_stream) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.iters):
                lib.roofprobe(v, ip, op, n, blocks, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            gbs = BYTES[v] * n / (ms * 1e-3) / 1e9
            res.append({"variant": v, "name": NAMES[v], "blocks": blocks, "ms": ms, "GBps": gbs})
            print(f"{NAMES[v]:28s} blocks={blocks:7d} {ms:8.3f} ms {gbs:8.1f} GB/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "roofprobe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
