#!/usr/bin/env python3
"""Run one native op on one shape repeatedly (for rocprofv3 --pmc passes and A/B timing).

    python tools/op_bench.py gemm_bn1 802816 256 64        # M N K  (A [M,K] x W[N,K]^T + BN stats)
    python tools/op_bench.py gemm 802816 256 64            # plain forward GEMM (GEMM_CFG=98: forced tile config)
    python tools/op_bench.py conv_fwd_bn 256 56 64 64 3 1  # N H C K R stride (pad R//2)
    python tools/op_bench.py conv_dgrad_bn 256 14 256 256 3 1
    python tools/op_bench.py conv_wgrad 256 14 256 256 3 1
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402


def main():
    op = sys.argv[1]
    a = [int(v) for v in sys.argv[2:]]
    iters = int(os.environ.get("ITERS", "20"))
    L = lib()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    if op in ("gemm", "gemm_bn1"):
        M, N, K = a
        A = torch.randn(M, K, device=dev, dtype=bf)
        W = torch.randn(N, K, device=dev, dtype=bf)
        out = torch.empty(M, N, device=dev, dtype=bf)
        fn = (lambda: L.gemm_bn(A, W, 1)) if op == "gemm_bn1" else (lambda: L.gemm(A, True, W, True, out, 1.0, 0.0,
                                                                                     None, 0, 1))
        fl = 2.0 * M * N * K
    elif op == "wgrad":  # dW[M,N] (+)= dY^T X: dY [K,M], X [K,N] both MN-contiguous, auto split-K, fp32 out
        M, N, K = a
        A = torch.randn(K, M, device=dev, dtype=bf)
        B = torch.randn(K, N, device=dev, dtype=bf)
        out = torch.zeros(M, N, device=dev, dtype=torch.float32)
        fn = lambda: L.gemm(A, False, B, False, out, 1.0, 1.0, None, 0, 0)  # noqa: E731
        fl = 2.0 * M * N * K
    elif op == "gemm_bn3":  # dgrad GEMM + BN backward partials, relu mask from packed bits, += into out
        M, N, K = a
        A = torch.randn(M, K, device=dev, dtype=bf)
        W = torch.randn(K, N, device=dev, dtype=bf)
        x = torch.randn(M, N, device=dev, dtype=bf)
        out = torch.randn(M, N, device=dev, dtype=bf)
        bits = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)
        ch = [torch.rand(N, device=dev) + 0.5 for _ in range(4)]
        fn = lambda: L.gemm_bn(A, W, 3, x, *ch, mask=bits, out=out)  # noqa: E731
        fl = 2.0 * M * N * K
    elif op in ("gemm_bn2",):
        M, N, K = a
        A = torch.randn(M, K, device=dev, dtype=bf)
        W = torch.randn(K, N, device=dev, dtype=bf)
        x = torch.randn(M, N, device=dev, dtype=bf)
        ch = [torch.rand(N, device=dev) + 0.5 for _ in range(4)]
        fn = lambda: L.gemm_bn(A, W, 2, x, *ch)  # noqa: E731
        fl = 2.0 * M * N * K
    else:
        N, H, C, K, R, st = a
        pad = R // 2
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, C, device=dev, dtype=bf)
        w = torch.randn(K, R, R, C, device=dev, dtype=bf)
        dy = torch.randn(N, P, P, K, device=dev, dtype=bf)
        fl = 2.0 * N * P * P * K * R * R * C
        if op == "conv_fwd_bn":
            fn = lambda: L.conv_fwd_bn(x, w, st, pad)  # noqa: E731
        elif op == "conv_fwd":
            fn = lambda: L.conv_fwd(x, w, st, pad)  # noqa: E731
        elif op == "conv_dgrad_bn":
            ch = [torch.rand(C, device=dev) + 0.5 for _ in range(4)]
            fn = lambda: L.conv_dgrad_bn(dy, w, H, H, st, pad, x.view(-1, C), *ch)  # noqa: E731
        elif op == "conv_dgrad":
            fn = lambda: L.conv_dgrad(dy, w, H, H, st, pad)  # noqa: E731
        elif op == "conv_wgrad":
            dw = torch.zeros(K, R, R, C, device=dev, dtype=torch.float32)
            fn = lambda: L.conv_wgrad(dy, x, dw, 1.0, st, pad)  # noqa: E731
        else:
            raise SystemExit(f"unknown op {op}")
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1e3
    print(f"{op} {a}: {us:.1f} us  {fl / us / 1e6:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
