#!/usr/bin/env python3
"""Experimental direct 3x3 conv from an LDS halo tile (csrc/lab/conv_halo.hip, lab extension) vs the implicit-GEMM conv
(conv_fwd / conv_fwd_bn) at ResNet-50's layer-1 shape: numerics against F.conv2d, then interleaved timing.

    python tools/conv_halo_ab.py [--batch 1024]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lab, lib  # noqa: E402


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
    a = ap.parse_args()
    L = lib()
    LAB = lab()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    # numerics at a small batch, with image edges in every band
    x = torch.randn(4, 56, 56, 64, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(dev, torch.bfloat16)
    y = LAB.conv_halo_fwd(x, w)[0]
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    rel = ((y.float() - ref).norm() / ref.norm()).item()
    y2 = L.conv_fwd(x, w, 1, 1)
    rel2 = ((y2.float() - ref).norm() / ref.norm()).item()
    print(f"numerics: halo rel err {rel:.2e}, implicit GEMM rel err {rel2:.2e}", flush=True)
    assert rel < 1e-2, rel
    N = a.batch
    x = torch.randn(N, 56, 56, 64, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * N * 56 * 56 * 64 * 64 * 9
    # at full size (more bands than CUs: the persistent form walks several per workgroup) against the GEMM
    yh, yg = LAB.conv_halo_fwd(x, w)[0].float(), L.conv_fwd(x, w, 1, 1).float()
    rel3 = ((yh - yg).norm() / yg.norm()).item()
    print(f"batch {N}: halo vs implicit GEMM rel diff {rel3:.2e}", flush=True)
    assert rel3 < 1e-2, rel3
    for r in range(2):
        th = timeit(lambda: LAB.conv_halo_fwd(x, w)[0])
        tg = timeit(lambda: L.conv_fwd(x, w, 1, 1))
        tb = timeit(lambda: L.conv_fwd_bn(x, w, 1, 1))
        ths = timeit(lambda: LAB.conv_halo_fwd(x, w, True))
        print(f"round {r}: halo {th:.1f} us ({fl / th / 1e6:.0f} TF/s)  implicit GEMM {tg:.1f} us  "
              f"| with BN stats: halo {ths:.1f} us  conv_fwd_bn {tb:.1f} us", flush=True)


if __name__ == "__main__":
    main()
