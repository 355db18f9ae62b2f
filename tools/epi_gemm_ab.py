#!/usr/bin/env python3
"""A/B of GEMM tile configurations WITH BERT's real epilogues (tools/gemm_ab.py times plain GEMMs only).

    python tools/epi_gemm_ab.py [--cfgs 0,1,25,29] [--rounds 3]

Cases (BERT-base, 32768 tokens):
  ffn1_fwd   f1 = gelu(x W1^T + b1), aux := gelu'(pre)        [32768 x 3072 x 768], aux mode 3
  ffn2_dgrad dpre = (df2 W2) * aux, colsum(dpre) -> db1         [32768 x 3072 x 768], aux mode 4 + column sums
  plain      the same shape, no epilogue
cfg 0 = dtg's heuristic; others: the forced table of csrc/kernels/gemm_forced*.hip.  Interleaved rounds in one
process; median us per call over ITERS calls of each round.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402
from _forced_gemm import forced_gemm  # noqa: E402


def timeit(fn, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0,1,25,29")
    ap.add_argument("--rounds", type=int, default=3)
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
    f1 = torch.empty(T, F, device=dev, dtype=bf)
    pre = torch.empty(T, F, device=dev, dtype=bf)
    dpre = torch.empty(T, F, device=dev, dtype=bf)
    gb1 = torch.zeros(F, device=dev)
    cases = {  # (the colsum epilogue of ffn2_dgrad is production-only: cfg 0)
        "ffn1_fwd": lambda c: forced_gemm(c, x, True, w1, True, f1, 1.0, 0.0, b1, 2, 0, pre, 3),
        "ffn2_dgrad": lambda c: L.gemm(df2, True, w2, False, dpre, 1.0, 0.0, None, 2, 0, pre, 4, colsum=gb1),
        "plain": lambda c: forced_gemm(c, x, True, w1, True, f1, 1.0, 0.0, None, 0, 0),
    }
    cfgs = [int(c) for c in a.cfgs.split(",")]
    res = {k: {c: [] for c in cfgs} for k in cases}
    for _ in range(a.rounds):
        for name, fn in cases.items():
            for c in cfgs:
                f = (lambda fn=fn, c=c: fn(c))
                f()
                res[name][c].append(timeit(f, a.iters))
    fl = 2.0 * T * F * H
    for name in cases:
        out = {str(c): {"us": round(sorted(v)[len(v) // 2], 1), "TF/s": round(fl / (sorted(v)[len(v) // 2] * 1e6), 1)}
               for c, v in res[name].items()}
        print(json.dumps({"case": name, **out}), flush=True)


if __name__ == "__main__":
    main()
