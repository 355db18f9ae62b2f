#!/usr/bin/env python3
"""The 1x1 stride-2 projection weight gradients of ResNet-50 at batch 1024, isolated: the implicit-GEMM conv wgrad
(conv.hip, strided gather) against a strided copy of x followed by the dense split-K GEMM wgrad the stride-1 1x1
convs use, both at the side-stream split target (256 workgroups).  Checks the two agree."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402
from dtg.ops.gemm import gemm  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
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
    L = lib()
    dev = torch.device("cuda")
    N = int(os.environ.get("BATCH", "1024"))
    for (H, C, K) in [(56, 256, 512), (28, 512, 1024), (14, 1024, 2048)]:
        g = torch.Generator(device="cpu").manual_seed(H)
        x4 = torch.randn(N, H, H, C, generator=g).to(dev, torch.bfloat16)
        dy4 = torch.randn(N, H // 2, H // 2, K, generator=g).to(dev, torch.bfloat16)
        dw_a = torch.zeros(K, 1, 1, C, device=dev)
        dw_b = torch.zeros(K, C, device=dev)
        P = N * (H // 2) ** 2
        sk = L.gemm_pick_split(K, C, P, False, 256)

        def implicit():
            L.conv_wgrad(dy4, x4, dw_a, 1.0, 2, 0, target_wgs=256)

        xs = torch.empty(N, H // 2, H // 2, C, device=dev, dtype=torch.bfloat16)

        def copy_gemm():
            xs.copy_(x4[:, ::2, ::2, :])
            gemm(dy4.view(P, K), False, xs.view(P, C), False, out=dw_b, beta=1.0, split_k=sk)

        def copy_only():
            xs.copy_(x4[:, ::2, ::2, :])

        r = {"x": [N, H, H, C], "K": K, "split": sk, "implicit_us": timeit(implicit), "copy_gemm_us": timeit(copy_gemm),
             "copy_us": timeit(copy_only)}
        dw_a.zero_()
        dw_b.zero_()
        implicit()
        copy_gemm()
        a, b = dw_a.view(K, C), dw_b
        r["rel_diff"] = float(((a - b).norm() / b.norm()).item())
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) and k != "rel_diff" else v) for k, v in r.items()}),
              flush=True)


if __name__ == "__main__":
    main()
