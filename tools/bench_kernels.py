#!/usr/bin/env python3
"""Kernel micro-benchmarks on the GPU: dtg's HIP kernels vs the vendor-library path torch uses
(hipBLASLt GEMM, MIOpen conv/BN), on the ResNet-50 / BERT-base shapes that matter.

    python tools/bench_kernels.py [--only gemm|bn|xent|optim] [--iters N]

Prints one line per case: time of each implementation, achieved TB/s (memory-bound view) and
TFLOP/s, and the speedup of dtg over the library.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dtg  # noqa: E402,F401
from dtg import ops  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def bench_gemm(iters, out):
    dev = "cuda"
    # (name, M, N, K, a_kc, b_kc)  -- ResNet-50 1x1 convs at batch 256 (fwd / dgrad / wgrad) + BERT
    cases = []
    for (hw, cin, cout) in [(56, 256, 64), (56, 64, 256), (28, 512, 128), (28, 128, 512), (14, 1024, 256),
                            (14, 256, 1024), (7, 2048, 512), (7, 512, 2048)]:
        M = 256 * hw * hw
        cases.append((f"r50 fwd {hw}x{hw} {cin}->{cout}", M, cout, cin, True, True))
        cases.append((f"r50 dgrad {hw}x{hw} {cin}->{cout}", M, cin, cout, True, False))
        cases.append((f"r50 wgrad {hw}x{hw} {cin}->{cout}", cout, cin, M, False, False))
    for (M, N, K) in [(16384, 2304, 768), (16384, 768, 768), (16384, 3072, 768), (16384, 768, 3072), (4096, 4096, 4096)]:
        cases.append((f"gemm {M}x{N}x{K}", M, N, K, True, True))
    # BERT-base backward at 8192 tokens: dgrad (B = W, MN-contiguous) and wgrad (both MN-contiguous)
    for (n_out, n_in) in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        cases.append((f"bert dgrad {n_out}->{n_in}", 8192, n_in, n_out, True, False))
        cases.append((f"bert wgrad {n_out}x{n_in}", n_out, n_in, 8192, False, False))
    for name, M, N, K, akc, bkc in cases:
        A = torch.randn((M, K) if akc else (K, M), device=dev, dtype=torch.bfloat16)
        B = torch.randn((N, K) if bkc else (K, N), device=dev, dtype=torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        Ct = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        At = A if akc else A.t()
        Bt = B.t() if bkc else B
        t_dtg = timeit(lambda: ops.gemm(A, akc, B, bkc, out=C), iters)
        t_lib = timeit(lambda: torch.matmul(At, Bt, out=Ct), iters)
        err = ((C.float() - Ct.float()).norm() / Ct.float().norm()).item()
        flops = 2.0 * M * N * K
        byts = 2.0 * (M * K + N * K + M * N)
        r = {"kind": "gemm", "case": name, "dtg_us": round(t_dtg, 1), "lib_us": round(t_lib, 1),
             "speedup": round(t_lib / t_dtg, 3), "dtg_tflops": round(flops / t_dtg / 1e6, 1),
             "dtg_TBps": round(byts / t_dtg / 1e6, 2), "rel_err": err}
        print(json.dumps(r), flush=True)
        out.append(r)


def bench_bn(iters, out):
    dev = "cuda"
    for (hw, c) in [(112, 64), (56, 64), (56, 256), (28, 128), (28, 512), (14, 256), (14, 1024), (7, 512), (7, 2048)]:
        x = torch.randn(256, c, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x)
        w = torch.ones(c, device=dev, requires_grad=True)
        b = torch.zeros(c, device=dev, requires_grad=True)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        xg = x.clone().requires_grad_()

        def dtg_fb():
            y = ops.batch_norm_act(xg, w, b, rm, rv, True, 0.1, 1e-5, r, True)
            y.backward(x)

        def lib_fb():
            y = F.relu(F.batch_norm(xg, rm, rv, w, b, True, 0.1, 1e-5) + r)
            y.backward(x)
        t_dtg = timeit(dtg_fb, iters)
        t_lib = timeit(lib_fb, iters)
        byts = x.numel() * 2 * 10.0  # ~10 tensor passes fwd+bwd with residual
        rr = {"kind": "bn_add_relu fwd+bwd", "case": f"{hw}x{hw}x{c}", "dtg_us": round(t_dtg, 1),
              "lib_us": round(t_lib, 1), "speedup": round(t_lib / t_dtg, 3), "dtg_TBps": round(byts / t_dtg / 1e6, 2)}
        print(json.dumps(rr), flush=True)
        out.append(rr)


def bench_xent(iters, out):
    dev = "cuda"
    for (B, V) in [(256, 1000), (4096, 30522)]:
        lg = torch.randn(B, V, device=dev, dtype=torch.bfloat16, requires_grad=True)
        lab = torch.randint(0, V, (B,), device=dev)

        def d():
            ops.softmax_cross_entropy(lg, lab).backward()

        def l():
            F.cross_entropy(lg, lab).backward()
        t_dtg, t_lib = timeit(d, iters), timeit(l, iters)
        r = {"kind": "softmax_xent fwd+bwd", "case": f"{B}x{V}", "dtg_us": round(t_dtg, 1), "lib_us": round(t_lib, 1),
             "speedup": round(t_lib / t_dtg, 3)}
        print(json.dumps(r), flush=True)
        out.append(r)


def bench_optim(iters, out):
    dev = "cuda"
    n = 25_600_000
    from dtg.ops import optim_kernels as K
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev, dtype=torch.bfloat16)
    m = torch.zeros(n, device=dev)
    mir = torch.empty(n, device=dev, dtype=torch.bfloat16)
    hyper = torch.tensor([0.1, 1.0], device=dev)
    t_dtg = timeit(lambda: K.momentum(w, g, m, hyper, mir, 0.9, 5e-5, False, 1.0, False), iters)
    params = [torch.randn(n // 160, device=dev, requires_grad=True) for _ in range(160)]
    for p in params:
        p.grad = torch.randn_like(p)
    opt = torch.optim.SGD(params, lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)
    t_lib = timeit(opt.step, iters)
    byts = n * (4 + 2 + 4 + 4 + 4 + 2)
    r = {"kind": "momentum-sgd apply", "case": "25.6M params", "dtg_us": round(t_dtg, 1),
         "lib_us(torch foreach fp32)": round(t_lib, 1), "speedup": round(t_lib / t_dtg, 3),
         "dtg_TBps": round(byts / t_dtg / 1e6, 2)}
    print(json.dumps(r), flush=True)
    out.append(r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = []
    for name, fn in [("gemm", bench_gemm), ("bn", bench_bn), ("xent", bench_xent), ("optim", bench_optim)]:
        if a.only in (None, name):
            fn(a.iters, out)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
