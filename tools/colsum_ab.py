#!/usr/bin/env python3
"""A/B: dgrad GEMM (aux-mode-4 GELU backward: x the saved GELU') + separate column-sum kernel vs the fused colsum epilogue."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402

L = lib()
dev = torch.device("cuda")
for M, N, K in [(32768, 3072, 768), (8192, 3072, 768)]:
    dy = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(K, N, device=dev) * 0.05).bfloat16()
    pre = torch.randn(M, N, device=dev).bfloat16()
    d = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev)
    fa = lambda: (L.gemm(dy, True, w, False, d, 1.0, 0.0, None, 2, 0, pre, 4), L.colsum(d, cs, True))  # noqa: E731
    fb = lambda: L.gemm(dy, True, w, False, d, 1.0, 0.0, None, 2, 0, pre, 4, colsum=cs)  # noqa: E731
    fc = lambda: L.gemm(dy, True, w, False, d, 1.0, 0.0, None, 2, 0, pre, 4)  # noqa: E731
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"sep": [], "fused": [], "gemm_only": []}
    for _ in range(5):
        for k, f in (("sep", fa), ("fused", fb), ("gemm_only", fc)):
            f()
            torch.cuda.synchronize()
            s.record()
            for _ in range(10):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) / 10 * 1e3)
    print(M, N, K, {k: round(sorted(v)[2], 1) for k, v in res.items()}, flush=True)
