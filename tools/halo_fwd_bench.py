#!/usr/bin/env python3
"""Isolated time of ResNet-50's stage-1 3x3 forward with BN statistics (conv_fwd_bn, 64 -> 64, 56x56, the direct
halo-tile kernel of csrc/kernels/conv_halo.hip) at the per-GPU batch; run under rocprofv3 for per-kernel counters.

    python tools/halo_fwd_bench.py [--n 1024] [--iters 20]
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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    L, dev = lib(), torch.device("cuda")
    x = torch.randn(a.n, 56, 56, 64, device=dev).bfloat16()
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).bfloat16()
    for _ in range(3):
        L.conv_fwd_bn(x, w, 1, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        L.conv_fwd_bn(x, w, 1, 1)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    fl = 2 * a.n * 56 * 56 * 64 * 64 * 9
    print(json.dumps({"n": a.n, "us": round(us, 1), "TFs": round(fl / us / 1e6, 1),
                      "TBs_x_plus_y": round(2 * x.numel() * 2 / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
