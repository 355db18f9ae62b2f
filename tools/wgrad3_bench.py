#!/usr/bin/env python3
"""Isolated time of ResNet-50's stride-1 3x3 weight gradients (conv_wgrad, dw fp32 += ) at the per-GPU batch, for
the split-K targets the model uses (models/resnet_fused.py): TFLOP/s and the operand bytes per call.

    python tools/wgrad3_bench.py [--n 1024] [--iters 20] [--targets 256,512]
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
    ap.add_argument("--targets", default="256,512")
    ap.add_argument("--stages", default="1,2,3,4", help="which of the four stages to time")
    ap.add_argument("--halo", type=int, default=1, help="conv_halo_wgrad_set value (stage 1: 0 implicit GEMM)")
    a = ap.parse_args()
    L, dev = lib(), torch.device("cuda")
    L.conv_halo_wgrad_set(a.halo)
    shapes = [(64, 56), (128, 28), (256, 14), (512, 7)]
    for c, h in [shapes[int(i) - 1] for i in a.stages.split(",")]:
        x = torch.randn(a.n, h, h, c, device=dev).bfloat16()
        dy = torch.randn(a.n, h, h, c, device=dev).bfloat16()
        dw = torch.zeros(c, 3, 3, c, device=dev)
        res = {}
        for t in map(int, a.targets.split(",")):
            for _ in range(3):
                L.conv_wgrad(dy, x, dw, 1.0, 1, 1, target_wgs=t)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                L.conv_wgrad(dy, x, dw, 1.0, 1, 1, target_wgs=t)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            fl = 2 * a.n * h * h * c * c * 9
            res[t] = {"us": round(us, 1), "TFs": round(fl / us / 1e6, 1),
                      "TBs_operands": round(2 * x.numel() * 2 / us / 1e6, 2)}
        print(json.dumps({"C": c, "H": h, "n": a.n, "by_target": res}), flush=True)
        del x, dy, dw


if __name__ == "__main__":
    main()
