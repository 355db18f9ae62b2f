#!/usr/bin/env python3
"""In-process A/B of GEMM tile configurations on given shapes (interleaved rounds, one process:
cdna_hip_programming.md §5.4 rule 24), against torch.matmul (hipBLASLt) on the same random data.

    python tools/gemm_ab.py --shapes 32768x3072x768,32768x768x3072 --cfgs 0,25,99 [--layout nn|nt|tn]

cfg 0 = dtg's heuristic, 25 = register-pipelined 128x128, 99 = 256x256 8-wave 8-phase (gemm8.hip);
the rest: csrc/kernels/gemm_forced.hip.  Layouts: A [M,K] K-contiguous with B [N,K] (fwd, "nt"),
B [K,N] (dgrad, "nn"); "tn": A stored [K,M] and B [K,N] (weight gradient, fp32 out).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", required=True)
    ap.add_argument("--cfgs", default="0,25,99")
    ap.add_argument("--layout", default="nt")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default="")
    ap.add_argument("--splits", default="0", help="comma list of split_k values to try (0 = heuristic)")
    ap.add_argument("--epi", default="none", choices=["none", "bias", "gelu", "dgelu"],
                    help="dtg epilogue: bias; bias + GELU with GELU' saved (BERT FFN1 forward); x saved GELU' "
                         "(FFN2 data gradient).  hipBLASLt ('lib') always runs the plain GEMM")
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    out = []
    for shp in a.shapes.split(","):
        M, N, K = (int(v) for v in shp.split("x"))
        g = torch.Generator(device="cpu").manual_seed(0)
        if a.layout == "tn":
            A = (torch.rand(K, M, generator=g) * 2 - 1).to(dev, torch.bfloat16)
            B = (torch.rand(K, N, generator=g) * 2 - 1).to(dev, torch.bfloat16)
            C = torch.zeros(M, N, device=dev, dtype=torch.float32)
            At, Bt, akc, bkc = A.t(), B, False, False
        else:
            A = (torch.rand(M, K, generator=g) * 2 - 1).to(dev, torch.bfloat16)
            if a.layout == "nt":
                B = (torch.rand(N, K, generator=g) * 2 - 1).to(dev, torch.bfloat16)
                Bt, bkc = B.t(), True
            else:
                B = (torch.rand(K, N, generator=g) * 2 - 1).to(dev, torch.bfloat16)
                Bt, bkc = B, False
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            At, akc = A, True
        Ct = torch.empty(M, N, device=dev, dtype=torch.bfloat16)  # hipBLASLt: bf16 out
        flops = 2.0 * M * N * K
        cfgs = [(int(c), int(sp)) for c in a.cfgs.split(",") for sp in a.splits.split(",")]
        bias = torch.randn(N, device=dev) if a.epi in ("bias", "gelu") else None
        aux = (torch.rand(M, N, device=dev) + 0.5).bfloat16() if a.epi in ("gelu", "dgelu") else None
        act, aux_mode = {"none": (0, 0), "bias": (0, 0), "gelu": (2, 3), "dgelu": (0, 4)}[a.epi]

        def run_cfg(cs):
            c, sp = cs
            forced_gemm(c, A, akc, B, bkc, C, 1.0, 0.0, bias, act, sp, aux, aux_mode)

        times = {c: [] for c in cfgs}
        times["lib"] = []
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for c in cfgs + ["lib"]:
                fn = (lambda: torch.matmul(At, Bt, out=Ct)) if c == "lib" else (lambda c=c: run_cfg(c))
                fn()
                torch.cuda.synchronize()
                s.record()
                for _ in range(a.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[c].append(s.elapsed_time(e) / a.iters * 1e3)
        res = {"shape": shp, "layout": a.layout}
        for c, ts in times.items():
            ts.sort()
            c = c if c == "lib" else (f"{c[0]}" if c[1] == 0 else f"{c[0]}/s{c[1]}")
            res[str(c)] = {"us_med": round(ts[len(ts) // 2], 1), "us_min": round(ts[0], 1),
                           "tflops": round(flops / ts[len(ts) // 2] / 1e6, 1)}
        # correctness of each dtg config against hipBLASLt
        ref = torch.matmul(At.float(), Bt.float()) if M * N * K <= 2 ** 36 and a.epi == "none" else None
        if ref is not None:
            for c in cfgs:
                run_cfg(c)
                key = f"{c[0]}" if c[1] == 0 else f"{c[0]}/s{c[1]}"
                res[key]["rel_err"] = float(((C.float() - ref).norm() / ref.norm()).item())
        print(json.dumps(res), flush=True)
        out.append(res)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
