#!/usr/bin/env python3
"""3x3 weight gradients of ResNet-50 stages 2-4 at batch 1024: the linear-halo kernel (csrc/kernels/conv_halo.hip,
conv3x3_lin_wgrad_kernel) vs the implicit-GEMM split-K wgrad (conv_lin_wgrad_set(0)), interleaved, with the
split-K reduce included (what conv_wgrad costs the step).

    python tools/conv_wgrad_ab.py [--batch 1024] [--rounds 2]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--shapes", default="28,14,7", help="comma-separated H (stage 2 = 28, 3 = 14, 4 = 7)")
    ap.add_argument("--only", choices=["lin", "implicit"], default=None, help="time one path only (profiling)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--target", type=int, default=0, help="implicit-GEMM split-K workgroup target (0 = default; "
                    "the ResNet step uses 256, DTG_RESNET_CWSPLIT_WGS)")
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    N = a.batch
    chans = {28: 128, 14: 256, 7: 512}
    for H in (int(v) for v in a.shapes.split(",")):
        C = chans[H]
        x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(C, 3, 3, C, device=dev)
        fl = 2.0 * N * H * H * C * C * 9

        def run(on):
            L.conv_lin_wgrad_set(on)
            try:
                L.conv_wgrad(dy, x, dw, 0.0, 1, 1, 0, a.target)
            finally:
                L.conv_lin_wgrad_set(1)
        if a.only:
            t = timeit(lambda: run(1 if a.only == "lin" else 0), a.iters)
            print(f"{H}x{H} x {C} {a.only}: {t:.1f} us ({fl / t / 1e6:.0f} TF/s)", flush=True)
            continue
        run(1)
        d1 = dw.clone()
        run(0)
        rel = ((d1 - dw).norm() / dw.norm()).item()
        print(f"{H}x{H} x {C}: lin vs implicit rel diff {rel:.2e}", flush=True)
        for r in range(a.rounds):
            t1 = timeit(lambda: run(1), a.iters)
            t0 = timeit(lambda: run(0), a.iters)
            print(f"  round {r}: lin-halo {t1:.1f} us ({fl / t1 / 1e6:.0f} TF/s)  implicit {t0:.1f} us "
                  f"({fl / t0 / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
