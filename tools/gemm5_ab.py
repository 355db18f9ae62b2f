#!/usr/bin/env python3
"""A/B of the GEMM lab v5 main loop (csrc/lab/gemm5.hip, dtg._lab) against dtg's production GEMM and hipBLASLt
(torch.matmul) on BERT-base's forward shapes, C = A B^T with A [M, K], B [N, K] bf16.

Interleaved rounds in one process on uniform random [-1, 1) operands; every candidate is checked against an
fp32 reference on 64 sampled rows.  Build the lab first: python tools/build_ext.py --only lab

    python tools/gemm5_ab.py [--rounds 5] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (M tokens, N out features, K)
    (32768, 3072, 768),   # BERT FFN1 forward
    (32768, 768, 3072),   # BERT FFN2 forward
    (32768, 2304, 768),   # BERT QKV
    (32768, 768, 768),    # BERT attention output
    (4096, 4608, 4096),   # square-ish
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import dtg  # noqa: F401
    from dtg.ops._native import lab as _lab_loader, lib
    lab = _lab_loader()
    L = lib()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (M, N, K) in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        bias = torch.rand(N, device=dev) - 0.5
        outs = {k: torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                for k in ("g5", "g5p", "dtg", "blas", "g5p_gelu", "dtg_gelu", "blas_gelu")}
        aux = {k: torch.empty(M, N, device=dev, dtype=torch.bfloat16) for k in ("g5p_gelu", "dtg_gelu")}
        cands = {
            "g5": lambda: lab.gemm5(A, B, outs["g5"], 1),
            "g5p": lambda: lab.gemm5p(A, B, outs["g5p"]),
            "dtg": lambda: L.gemm(A, True, B, True, outs["dtg"]),
            "blas": lambda: torch.matmul(A, B.t(), out=outs["blas"]),
            # the BERT FFN1 forward epilogue: + bias, GELU, GELU'(pre) saved for the backward (dtg), or not (blas)
            "g5p_gelu": lambda: lab.gemm5p(A, B, outs["g5p_gelu"], bias, 2, aux["g5p_gelu"], 3),
            "dtg_gelu": lambda: L.gemm(A, True, B, True, outs["dtg_gelu"], 1.0, 0.0, bias, 2, 0, aux["dtg_gelu"], 3),
            # (hipBLASLt's fused bias + GELU kernel; the result is a fresh tensor from the caching allocator -- an
            # earlier version copied it into outs["blas_gelu"], which added a 201 MB copy to hipBLASLt's time)
            "blas_gelu": lambda: outs.__setitem__("blas_gelu", torch._addmm_activation(bias.bfloat16(), A, B.t(),
                                                                                        use_gelu=True)),
        }
        rows = torch.randint(0, M, (64,), device=dev)
        ref = A[rows].float() @ B.float().t()
        refg = torch.nn.functional.gelu(ref + bias, approximate="tanh")
        errs = {}
        for k, fn in cands.items():
            fn()
            torch.cuda.synchronize()
            r = refg if k.endswith("gelu") else ref
            errs[k] = ((outs[k][rows].float() - r).norm() / r.norm()).item()
        times = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                fn()
                s.record()
                for _ in range(a.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[k].append(s.elapsed_time(e) / a.iters * 1e3)
        flop = 2.0 * M * N * K
        res = {k: {"us": round(sorted(v)[len(v) // 2], 1), "TFs": round(flop / sorted(v)[len(v) // 2] / 1e6, 1),
                   "rel_err": float("%.3g" % errs[k])} for k, v in times.items()}
        print(json.dumps({"shape": [M, N, K], **res}), flush=True)

if __name__ == "__main__":
    main()
