#!/usr/bin/env python3
"""BERT FFN2 data gradient (dpre = (df2 W2) * GELU'(pre), + db1 column sums: the mode-5 BN-epilogue GEMM) under
each forced tile of gemm_bn_force_cfg (0 = heuristic, 1 128x128, 2 64x256, 3 128x128 register-pipelined, 4 256x64,
5 128x256 8 waves, 6 256x128 8 waves), interleaved rounds, median us.

    python tools/bn5_cfg_ab.py [--rounds 5]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    T, H, F = 32768, 768, 3072
    g = torch.Generator(device="cpu").manual_seed(0)
    w2 = (torch.rand(H, F, generator=g) * 0.1 - 0.05).to(dev, torch.bfloat16)
    df2 = (torch.rand(T, H, generator=g) * 2 - 1).to(dev, torch.bfloat16)
    pre = (torch.rand(T, F, generator=g) + 0.5).to(dev, torch.bfloat16)
    out = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
    gb1 = torch.zeros(F, device=dev)
    ref = None
    times = {c: [] for c in range(7)}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for c in times:
            L.gemm_bn_force_cfg(c)
            fn = lambda: L.gemm(df2, True, w2, False, out, 1.0, 0.0, None, 2, 0, pre, 4, colsum=gb1)  # noqa: E731
            fn()
            if ref is None:
                torch.cuda.synchronize()
                ref = out.float().clone()
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[c].append(s.elapsed_time(e) / a.iters * 1e3)
            err = ((out.float() - ref).norm() / ref.norm()).item()
            assert err < 1e-6, (c, err)
    L.gemm_bn_force_cfg(0)
    print(json.dumps({str(c): round(sorted(v)[len(v) // 2], 1) for c, v in times.items()}), flush=True)


if __name__ == "__main__":
    main()
