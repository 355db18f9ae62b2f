"""Isolated timing of the fused stem BN + ReLU + max-pool kernels (csrc/kernels/stem.hip) at ResNet-50's
stem shape: forward with / without saving y at the argmax, backward with the pooled-resolution statistics
pass / the pixel-resolution banded pass.  python tools/stem_ab.py [--batch 1024] [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    N, H, C = a.batch, 112, 64
    y = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    yf = y.float().reshape(-1, C)
    part = torch.zeros(32, 2, C, device=dev)
    part[0, 0] = yf.sum(0)
    part[0, 1] = (yf * yf).sum(0)
    del yf
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.rand(C, device=dev) - 0.5
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    res = {}
    for yam in (False, True):
        res[yam] = L.stem_bn_pool_fwd(y, part, gamma, beta, rm, rv, 0.1, 1e-5, 3, 2, 1, save_yam=yam)
        t = _time(lambda: L.stem_bn_pool_fwd(y, part, gamma, beta, rm, rv, 0.1, 1e-5, 3, 2, 1, save_yam=yam),
                  a.iters)
        print(f"fwd save_yam={int(yam)}: {t:.1f} us", flush=True)
    out, idx, smean, sinv, ym = res[True]
    dout = torch.randn_like(out.float()).to(torch.bfloat16)
    for yam in (None, ym):
        t = _time(lambda: L.stem_bn_pool_bwd(dout, idx, y, gamma, beta, smean, sinv, 3, 2, 1, yam=yam), a.iters)
        print(f"bwd pooled_stats={int(yam is not None)}: {t:.1f} us", flush=True)
    d0 = L.stem_bn_pool_bwd(dout, idx, y, gamma, beta, smean, sinv, 3, 2, 1)
    d1 = L.stem_bn_pool_bwd(dout, idx, y, gamma, beta, smean, sinv, 3, 2, 1, yam=ym)
    for n, u, v in zip(("dy", "dgamma", "dbeta"), d0, d1):
        u, v = u.float(), v.float()
        print(f"{n}: rel diff {((u - v).norm() / u.norm()).item():.2e}", flush=True)


if __name__ == "__main__":
    main()
