#!/usr/bin/env python3
"""Where does the BERT FFN1 forward epilogue's time go?  The 32768x3072x768 GEMM (x W1^T) timed with epilogues that
add one cost at a time: the bias, a second 201 MB output (aux mode 1: the pre-activation), the GELU arithmetic
(act 2), and the full FFN1 epilogue (bias + GELU + GELU'(pre) saved, aux mode 3); and the FFN2 data gradient
(df2 W2, 32768x3072x768 NN) plain, x saved GELU' (aux mode 4), and + the db1 column sums.  Interleaved rounds in
one process, median us.

    python tools/epi_decomp.py [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    T, H, F = 32768, 768, 3072
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.rand(T, H, generator=g) * 2 - 1).to(dev, bf)
    w1 = (torch.rand(F, H, generator=g) * 0.1 - 0.05).to(dev, bf)
    b1 = torch.rand(F, generator=g).to(dev) * 0.1
    w2 = (torch.rand(H, F, generator=g) * 0.1 - 0.05).to(dev, bf)
    df2 = (torch.rand(T, H, generator=g) * 2 - 1).to(dev, bf)
    out = torch.empty(T, F, device=dev, dtype=bf)
    aux = (torch.rand(T, F, generator=g) + 0.5).to(dev, bf)
    gb1 = torch.zeros(F, device=dev)
    cases = {
        "fwd plain": lambda: L.gemm(x, True, w1, True, out),
        "fwd +bias": lambda: L.gemm(x, True, w1, True, out, 1.0, 0.0, b1, 0, 0),
        "fwd +bias +aux store (no GELU)": lambda: L.gemm(x, True, w1, True, out, 1.0, 0.0, b1, 0, 0, aux, 1),
        "fwd +bias +GELU (one output)": lambda: L.gemm(x, True, w1, True, out, 1.0, 0.0, b1, 2, 0),
        "fwd +bias +GELU +GELU' saved": lambda: L.gemm(x, True, w1, True, out, 1.0, 0.0, b1, 2, 0, aux, 3),
        "dgrad plain": lambda: L.gemm(df2, True, w2, False, out),
        "dgrad x aux": lambda: L.gemm(df2, True, w2, False, out, 1.0, 0.0, None, 2, 0, aux, 4),
        "dgrad x aux +colsum": lambda: L.gemm(df2, True, w2, False, out, 1.0, 0.0, None, 2, 0, aux, 4, colsum=gb1),
    }
    times = {k: [] for k in cases}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for k, fn in cases.items():
            fn()
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / a.iters * 1e3)
    fl = 2.0 * T * F * H
    for k, v in times.items():
        v.sort()
        print(json.dumps({"case": k, "us": round(v[len(v) // 2], 1), "TF/s": round(fl / v[len(v) // 2] / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
