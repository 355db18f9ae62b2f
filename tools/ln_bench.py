#!/usr/bin/env python3
"""Time dtg's LayerNorm forward / backward kernels at a BERT shape (HIP events, median of ITERS).

    python tools/ln_bench.py [T=32768] [H=768]

Prints one JSON line per case with us per call and the effective HBM rate of the bytes the kernel must
move (bf16 activations in/out; the per-block parameter partials are not counted).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return t[len(t) // 2]


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    iters = int(os.environ.get("ITERS", "50"))
    L = lib()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    h = torch.randn(T, H, device=dev, dtype=bf)
    res = torch.randn(T, H, device=dev, dtype=bf)
    g = torch.rand(H, device=dev) + 0.5
    b = torch.randn(H, device=dev)
    y, s, mean, rstd = L.ln_fwd(h, res, g, b, 1e-12, 0.1, 7, 0.0, 0, True)
    dy = torch.randn(T, H, device=dev, dtype=bf)
    gg, gb, gz = (torch.zeros(H, device=dev) for _ in range(3))
    mb = T * H * 2 / 1e6
    cases = [
        ("ln_fwd res+dropout", lambda: L.ln_fwd(h, res, g, b, 1e-12, 0.1, 7, 0.0, 0, True), 4 * mb),
        ("ln_bwd dropout+dh+dbias", lambda: L.ln_bwd(dy, s, g, mean, rstd, gg, gb, 0.1, 7, 0.0, 0, True, gz), 4 * mb),
        ("ln_bwd plain", lambda: L.ln_bwd(dy, s, g, mean, rstd, gg, gb, 0.0, 0, 0.0, 0, False), 3 * mb),
    ]
    for name, fn, mbytes in cases:
        us = timeit(fn, iters)
        print(json.dumps({"case": name, "T": T, "H": H, "us": round(us, 1), "TB/s": round(mbytes / us, 2)}), flush=True)


if __name__ == "__main__":
    main()
