#!/usr/bin/env python3
"""BN-epilogue GEMMs at the ResNet-50 b512 1x1-conv shapes under the tile configuration forced by
``--cfg`` (lib().gemm_bn_force_cfg, csrc/kernels/gemm.hip gemm_bn_dispatch; 0 = heuristic).  One JSON line per case:
us per call and the rate over the compulsory HBM bytes.

    for c in 0 1 2 3 4 5 6; do python tools/bn_gemm_ab.py --cfg $c; done
    python tools/bn_gemm_ab.py --batch 1024 ... (the same shapes at per-GPU batch 1024)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402

# (mode, M, N, K): mode 1 = forward 1x1 conv + BN statistics (A [M,K] x W[N,K]^T); mode 3 = dgrad of the
# next block's conv1 + BN3 backward partials + relu mask bits + residual gradient accumulated in place;
# mode 2 = dgrad + BN backward with the mask recomputed from x
CASES = [(1, 1605632, 256, 64), (1, 401408, 512, 128), (1, 100352, 1024, 256), (1, 25088, 2048, 512),
         (1, 1605632, 64, 256), (1, 401408, 128, 512), (1, 100352, 256, 1024), (1, 25088, 512, 2048),
         (3, 1605632, 256, 64), (3, 401408, 512, 128), (3, 100352, 1024, 256), (3, 25088, 2048, 512),
         (2, 1605632, 64, 256), (2, 401408, 128, 512), (2, 100352, 256, 1024), (2, 25088, 512, 2048)]


def timeit(fn, iters=10):
    for _ in range(2):
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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--plain", action="store_true", help="also time the plain GEMM (no BN epilogue) per case")
    ap.add_argument("--modes", default="1,2,3")
    a = ap.parse_args()
    modes = {int(m) for m in a.modes.split(",")}
    L = lib()
    L.gemm_bn_force_cfg(a.cfg)
    dev = torch.device("cuda")
    bf = torch.bfloat16
    cfg = str(a.cfg)
    scale = a.batch // 512  # CASES are ResNet-50 b512 shapes
    for mode, M, N, K in CASES:
        if mode not in modes:
            continue
        M *= scale
        A = torch.randn(M, K, device=dev, dtype=bf)
        ch = [torch.rand(N, device=dev) + 0.5 for _ in range(4)]
        if mode == 1:
            W = torch.randn(N, K, device=dev, dtype=bf)
            fn = lambda: L.gemm_bn(A, W, 1)  # noqa: E731
            nbytes = 2 * (M * K + M * N)
        else:
            W = torch.randn(K, N, device=dev, dtype=bf)
            x = torch.randn(M, N, device=dev, dtype=bf)
            if mode == 3:
                out = torch.randn(M, N, device=dev, dtype=bf)
                bits = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)
                fn = lambda: L.gemm_bn(A, W, 3, x, *ch, mask=bits, out=out)  # noqa: E731
                nbytes = 2 * (M * K + 3 * M * N) + M * N // 8
            else:
                fn = lambda: L.gemm_bn(A, W, 2, x, *ch)  # noqa: E731
                nbytes = 2 * (M * K + 2 * M * N)
        us = timeit(fn)
        rec = {"cfg": int(cfg), "mode": mode, "M": M, "N": N, "K": K, "us": round(us, 1),
               "TBps": round(nbytes / us / 1e6, 2), "TFps": round(2.0 * M * N * K / us / 1e6, 1)}
        if a.plain:
            Wp = torch.randn(N, K, device=dev, dtype=bf)
            C = torch.empty(M, N, device=dev, dtype=bf)
            rec["plain_us"] = round(timeit(lambda: L.gemm(A, True, Wp, True, C, 1.0, 0.0, None, 0, 1)), 1)
            rec["lib_us"] = round(timeit(lambda: torch.matmul(A, Wp.t(), out=C)), 1)
            del Wp, C
        print(json.dumps(rec), flush=True)
        del A, W


if __name__ == "__main__":
    main()
