#!/usr/bin/env python3
"""Calibration only: does the relative placement of the 10 SoA streams (6 in, 4 out) change the HBM
rate of the eval+pdf access pattern?  The streams are carved from one allocation with a stride of
n*4 + pad bytes; pad sweeps 0 .. 2 MiB.  Uses tools/libroofprobe.so variants 1 (nt) and 6."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libroofprobe.so"))
    lib.roofprobe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                              ctypes.c_void_p]
    n = 100_000_000
    s = torch.cuda.current_stream()
    for pad in (0, 256, 4096, 65536, 65536 + 4096, 1 << 20, (1 << 20) + 12288, 2 << 20):
        stride = n + pad // 4                     # floats
        buf = torch.rand(10 * stride + 64, device="cuda")
        base = buf.data_ptr()
        ptrs = [base + 4 * k * stride for k in range(10)]
        in_ptrs = (ctypes.c_void_p * 6)(*ptrs[:6])
        out_ptrs = (ctypes.c_void_p * 4)(*ptrs[6:])
        for v in (1, 6):
            blocks = (n // 4 + 255) // 256 if v == 1 else (n // 4 + 511) // 512
            for _ in range(3):
                assert lib.roofprobe(v, in_ptrs, out_ptrs, n, blocks, s.cuda_stream) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                lib.roofprobe(v, in_ptrs, out_ptrs, n, blocks, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(f"pad={pad:8d} variant={v} {ms:.3f} ms {40 * n / (ms * 1e-3) / 1e9:.1f} GB/s", flush=True)
        del buf


if __name__ == "__main__":
    main()
