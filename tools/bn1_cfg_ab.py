#!/usr/bin/env python3
"""Forward BN-statistics GEMMs (gemm_bn mode 1) of ResNet-50 at per-GPU batch 1024 under every forced tile
(gemm_bn_force_cfg: 0 heuristic, 1 128x128, 2 64x256, 3 128x128 register-pipelined, 4 256x64, 5 128x256 8 waves,
6 256x128 8 waves), interleaved in one process, median us.

    python tools/bn1_cfg_ab.py [--rounds 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402

SHAPES = [(200704, 1024, 256), (50176, 2048, 512), (200704, 256, 1024), (50176, 512, 2048), (802816, 128, 512),
          (3211264, 64, 256), (802816, 256, 256), (200704, 512, 512), (50176, 1024, 1024)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for (M, N, K) in SHAPES:
        A = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
        times = {c: [] for c in range(7)}
        for _ in range(a.rounds):
            for c in times:
                L.gemm_bn_force_cfg(c)
                L.gemm_bn(A, W, 1)
                s.record()
                for _ in range(a.iters):
                    L.gemm_bn(A, W, 1)
                e.record()
                torch.cuda.synchronize()
                times[c].append(s.elapsed_time(e) / a.iters * 1e3)
        L.gemm_bn_force_cfg(0)
        print(json.dumps({"shape": [M, N, K], **{str(c): round(sorted(v)[len(v) // 2], 1) for c, v in times.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
