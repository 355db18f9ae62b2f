#!/usr/bin/env python3
"""Isolated time of ResNet-50's stage-1 3x3 data gradient with the BN-backward mode-3 epilogue (conv_dgrad_bn with
packed mask bits, 64 -> 64, 56x56): the direct halo-tile kernel (csrc/kernels/conv_halo.hip, EPI 1) against the
implicit-GEMM dgrad (conv_halo_dgrad_set(0)).

    python tools/halo_dgrad_ab.py [--n 1024] [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    L, dev, C, H = lib(), torch.device("cuda"), 64, 56
    w = (torch.randn(C, 3, 3, C, device=dev) * (9 * C) ** -0.5).bfloat16()
    dy = torch.randn(a.n, H, H, C, device=dev).bfloat16()
    x = torch.randn(a.n * H * H, C, device=dev).bfloat16()
    mean, inv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    bits = torch.randint(0, 256, (a.n * H * H, C // 8), device=dev, dtype=torch.uint8)
    res = {}
    for halo in (0, 1, 0, 1):
        L.conv_halo_dgrad_set(halo)
        for _ in range(5):
            L.conv_dgrad_bn(dy, w, H, H, 1, 1, x, mean, inv, gamma, beta, bits=bits)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            L.conv_dgrad_bn(dy, w, H, H, 1, 1, x, mean, inv, gamma, beta, bits=bits)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        res.setdefault("halo" if halo else "implicit", []).append(round(us, 1))
    L.conv_halo_dgrad_set(1)
    flops = 2 * a.n * H * H * C * C * 9
    print(json.dumps({"n": a.n, "us": res, "TFs_best": {k: round(flops / min(v) / 1e6, 1) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
