#!/usr/bin/env python3
"""Production halo-tile 3x3 forward with BN statistics (csrc/kernels/conv_halo.hip, conv_fwd_bn) vs the implicit-GEMM
conv (conv_halo_fwd_set(0)) at ResNet-50's stage-1 shape: numerics against F.conv2d, then interleaved timing.

    python tools/conv_halo_ab.py [--batch 1024]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

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


def fwd(L, x, w, halo):
    L.conv_halo_fwd_set(halo)
    try:
        return L.conv_fwd_bn(x, w, 1, 1)
    finally:
        L.conv_halo_fwd_set(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 56, 56, 64, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(dev, torch.bfloat16)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    for halo in (1, 0):
        rel = ((fwd(L, x, w, halo)[0].float() - ref).norm() / ref.norm()).item()
        print(f"numerics ({'halo' if halo else 'implicit GEMM'}): rel err {rel:.2e}", flush=True)
        assert rel < 1e-2, rel
    N = a.batch
    x = torch.randn(N, 56, 56, 64, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * N * 56 * 56 * 64 * 64 * 9
    yh, yg = fwd(L, x, w, 1)[0].float(), fwd(L, x, w, 0)[0].float()
    rel3 = ((yh - yg).norm() / yg.norm()).item()
    print(f"batch {N}: halo vs implicit GEMM rel diff {rel3:.2e}", flush=True)
    assert rel3 < 1e-2, rel3
    for r in range(2):
        th = timeit(lambda: fwd(L, x, w, 1))
        tg = timeit(lambda: fwd(L, x, w, 0))
        print(f"round {r}: conv_fwd_bn halo {th:.1f} us ({fl / th / 1e6:.0f} TF/s)  implicit GEMM {tg:.1f} us "
              f"({fl / tg / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
