#!/usr/bin/env python3
"""Tile-configuration sweep of the MFMA GEMM on the ResNet-50 / BERT shapes (production heuristic = cfg 0, forced tiles through the lab extension, tools/_forced_gemm.py):
one line per (shape, config) with time, TB/s and TFLOP/s; the fastest config per shape is marked.
This is the data the heuristic in csrc/kernels/gemm.hip (gemm_bf16) is fitted to.

    python tools/gemm_sweep.py [--json out.json] [--cfgs 0,1,2,...]
Configs: 0 heuristic, 1-4 128x128 S=1..4, 5-7 256x64 S=2..4, 8 256x128x3 (8 waves),
9 256x128x2 (8w), 10 128x256x2 (8w), 11 128x256x3 (8w), 12-13 64x256 S=2..3, 99 8-phase 256x256.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402
from _forced_gemm import forced_gemm  # noqa: E402

NAMES = {0: "heur", 1: "128x128s1", 2: "128x128s2", 3: "128x128s3", 4: "128x128s4", 5: "256x64s2", 6: "256x64s3",
         7: "256x64s4", 8: "256x128s3w8", 9: "256x128s2w8", 10: "128x256s2w8", 11: "128x256s3w8", 12: "64x256s2",
         13: "64x256s3", 14: "256x64s1", 15: "64x256s1", 16: "128x128s2k32",
         17: "128x128s3k32", 18: "128x128s4k32", 19: "64x256s3k32", 20: "256x64s3k32", 21: "64x256s2k32",
         22: "256x64s2k32", 23: "128x128s5k32", 24: "64x256s4k32", 25: "128x128s1rp", 26: "64x256s1rp", 27: "256x64s1rp",
         99: "8phase"}

# (M, N, K, a_kc, b_kc, beta): the memory-bound and mid-size GEMMs of a ResNet-50 batch-256 step
SHAPES = [
    (802816, 64, 256, True, True, 0.0), (802816, 256, 64, True, True, 0.0), (802816, 256, 64, True, False, 1.0),
    (802816, 64, 256, True, False, 0.0), (200704, 128, 512, True, True, 0.0), (200704, 512, 128, True, True, 0.0),
    (200704, 512, 128, True, False, 1.0), (50176, 1024, 256, True, True, 0.0), (50176, 1024, 256, True, False, 1.0),
    (50176, 256, 1024, True, True, 0.0), (12544, 2048, 512, True, True, 0.0), (12544, 512, 2048, True, True, 0.0),
    (200704, 256, 512, True, True, 0.0), (802816, 128, 256, True, True, 0.0),
    (16384, 768, 3072, True, True, 0.0), (16384, 3072, 768, True, True, 0.0), (16384, 2304, 768, True, True, 0.0),
    # weight gradients dW = dY^T X (both operands MN-contiguous, K = batch*H*W, auto split-K)
    (64, 256, 802816, False, False, 1.0), (256, 64, 802816, False, False, 1.0), (128, 512, 200704, False, False, 1.0),
    (512, 128, 200704, False, False, 1.0), (256, 1024, 50176, False, False, 1.0), (1024, 256, 50176, False, False, 1.0),
    (2048, 512, 12544, False, False, 1.0),
    # BERT-base weight gradients (tokens = 64 x 128)
    (768, 3072, 8192, False, False, 1.0), (3072, 768, 8192, False, False, 1.0), (2304, 768, 8192, False, False, 1.0),
    (768, 768, 8192, False, False, 1.0),
    # BERT-base batch 64 x 128 forward / data-gradient GEMMs (B = W as [out, in]: KC forward, MC dgrad)
    (8192, 768, 3072, True, False, 0.0), (8192, 768, 2304, True, False, 0.0), (8192, 3072, 768, True, False, 0.0),
    (8192, 768, 3072, True, True, 0.0), (8192, 3072, 768, True, True, 0.0), (8192, 2304, 768, True, True, 0.0),
    (8192, 768, 768, True, True, 0.0),
]


def timeit(fn, iters=10, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    ap.add_argument("--cfgs", default="0,1,2,3,14,15,16,17,18,19,20,21,22,23,24")
    ap.add_argument("--shapes", default="", help="comma list of shape indices (default all)")
    ap.add_argument("--splits", default="", help="comma list of split-K counts to force (0 = auto)")
    a = ap.parse_args()
    L = lib()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    res = []
    idx = [int(i) for i in a.shapes.split(",")] if a.shapes else range(len(SHAPES))
    for (M, N, K, akc, bkc, beta) in [SHAPES[i] for i in idx]:
        splits = [int(v) for v in a.splits.split(",")] if a.splits else [0 if K >= 8192 else 1]
        A = torch.randn((M, K) if akc else (K, M), device="cuda", dtype=torch.bfloat16)
        B = torch.randn((N, K) if bkc else (K, N), device="cuda", dtype=torch.bfloat16)
        C = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        ref = None
        by = (A.numel() + B.numel()) * 2 + C.numel() * 2 * (2 if beta else 1)
        fl = 2.0 * M * N * K
        rows = []
        for c in cfgs:
            if c in (5, 6, 7, 14, 20, 22, 27) and N > 64 and N % 64:
                continue
            for split in splits:
                out = torch.zeros_like(C)
                forced_gemm(c, A, akc, B, bkc, out, 1.0, 0.0, None, 0, split)
                if ref is None:
                    ref = out.float()
                err = ((out.float() - ref).norm() / (ref.norm() + 1e-9)).item()
                us = timeit(lambda: forced_gemm(c, A, akc, B, bkc, C, 1.0, beta, None, 0, split))
                rows.append((c if len(splits) == 1 else (c, split), us, err))
        best = min(r[1] for r in rows)
        for c, us, err in rows:
            mark = " *" if us == best else ""
            name = NAMES[c] if isinstance(c, int) else f"{NAMES[c[0]]}/split{c[1]}"
            print(f"{M:7d}x{N:5d}x{K:5d} {'KC' if akc else 'MC'}{'KC' if bkc else 'MC'} b={beta:.0f} "
                  f"{name:18s} {us:8.1f} us {by / us / 1e6:5.2f} TB/s {fl / us / 1e6:6.1f} TF/s err={err:.1e}{mark}",
                  flush=True)
            res.append({"M": M, "N": N, "K": K, "akc": akc, "bkc": bkc, "beta": beta, "cfg": name, "us": us,
                        "err": err})
        del A, B, C
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
