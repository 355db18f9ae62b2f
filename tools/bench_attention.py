#!/usr/bin/env python3
"""Attention microbenchmark at the BERT-base shape: fused kernels (attention.hip) vs the unfused
path (strided-batched MFMA GEMMs + softmax kernels)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops import lib, transformer as T  # noqa: E402


def timeit(fn, iters=20):
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
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--nh", type=int, default=12)
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    B, S, nh = a.B, a.S, a.nh
    H = nh * 64
    qkv = torch.randn(B * S, 3 * H, device="cuda").bfloat16()
    mask = torch.zeros(B, S, device="cuda")
    dout = torch.randn(B * S, H, device="cuda").bfloat16()
    L = lib()
    out, lse = L.attn_fused_fwd(qkv, mask, B, S, nh, a.p, 1)
    r = {"shape": [B, S, nh]}
    r["fused_fwd_us"] = timeit(lambda: L.attn_fused_fwd(qkv, mask, B, S, nh, a.p, 1))
    r["fused_bwd_us"] = timeit(lambda: L.attn_fused_bwd(qkv, out, dout, lse, mask, B, S, nh, a.p, 1))
    cx, P, Pd = T.attention_fwd(qkv, mask, B, S, nh, a.p, 1)
    dq = torch.empty_like(qkv)
    r["gemm_fwd_us"] = timeit(lambda: T.attention_fwd(qkv, mask, B, S, nh, a.p, 1))
    r["gemm_bwd_us"] = timeit(lambda: T.attention_bwd(dout, qkv, P, Pd, B, S, nh, dq))
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
