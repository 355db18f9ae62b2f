#!/usr/bin/env python3
"""Per-tile error map of the persistent v5 GEMM (dtg._lab.gemm5p) at a forced grid: which (tile, position in the
workgroup's tile sequence) is wrong.  Tile t runs on workgroup t % G as its (t // G)-th tile."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import dtg  # noqa: F401
    from dtg.ops._native import lab
    dev = torch.device("cuda")
    for (M, N, K, G) in [(2048, 768, 768, 4), (2048, 768, 128, 4), (2048, 768, 64, 4), (1024, 384, 192, 2)]:
        torch.manual_seed(0)
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        assert lab().gemm5p(A, B, out, grid=G)
        torch.cuda.synchronize()
        ref = A.float() @ B.float().t()
        tn = N // 192
        errs = {}
        for t in range((M // 256) * tn):
            bm, bn = (t // tn) * 256, (t % tn) * 192
            o, r = out[bm:bm + 256, bn:bn + 192].float(), ref[bm:bm + 256, bn:bn + 192]
            errs[t] = round(((o - r).norm() / r.norm()).item(), 4)
        by_pos = {}
        for t, e in errs.items():
            by_pos.setdefault(t // G, []).append(e)
        print(json.dumps({"M": M, "N": N, "K": K, "G": G, "err_by_seq_pos": {k: max(v) for k, v in by_pos.items()}}),
              flush=True)
        if max(errs.values()) > 0.01:
            t = max(errs, key=errs.get)
            bm, bn = (t // tn) * 256, (t % tn) * 192
            d = (out[bm:bm + 256, bn:bn + 192].float() - ref[bm:bm + 256, bn:bn + 192]).abs()
            rows = (d.max(1).values > 0.5).nonzero().flatten().tolist()
            cols = (d.max(0).values > 0.5).nonzero().flatten().tolist()
            print(json.dumps({"worst_tile": t, "bad_rows": rows[:40], "n_bad_rows": len(rows), "bad_cols": cols[:40],
                              "n_bad_cols": len(cols)}), flush=True)


if __name__ == "__main__":
    main()
