#!/usr/bin/env python3
"""Bandwidth of dtg's BatchNorm streaming passes at the ResNet-50 b512 shapes vs a plain PyTorch
elementwise pass that moves the same bytes (torch.add of two bf16 tensors: read 2, write 1).

    python tools/bn_bench.py [--iters 20]

Rows: bn_fwd_part (BN apply + residual + relu + packed mask bits; finalize included) and bn_bwd_part
(dx pass; finalize included), each with its achieved TB/s over its compulsory bytes."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402

SHAPES = [(1605632, 256), (1605632, 64), (401408, 512), (401408, 128), (100352, 1024), (100352, 256)]


def timeit(fn, iters):
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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    out = []
    for M, C in SHAPES:
        x = torch.randn(M, C, device=dev).bfloat16()
        r = torch.randn(M, C, device=dev).bfloat16()
        g = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        part = L.bn_part_alloc(x, C, False)
        bits = torch.empty(M, C // 8, device=dev, dtype=torch.uint8)
        nb = x.numel() * 2
        res = {"shape": [M, C]}
        us = timeit(lambda: torch.add(x, r), a.iters)
        res["torch_add_us"], res["torch_add_TBps"] = round(us, 1), round(3 * nb / us / 1e6, 2)
        us = timeit(lambda: L.bn_fwd_part(x, part, r, g, b, rm, rv, 0.1, 1e-5, True, bits=bits), a.iters)
        res["apply_res_us"], res["apply_res_TBps"] = round(us, 1), round((3 * nb + nb // 16) / us / 1e6, 2)
        us = timeit(lambda: L.bn_fwd_part(x, part, None, g, b, rm, rv, 0.1, 1e-5, True, bits=bits), a.iters)
        res["apply_us"], res["apply_TBps"] = round(us, 1), round((2 * nb + nb // 16) / us / 1e6, 2)
        us = timeit(lambda: L.bn_fwd_part(x, part, None, g, b, rm, rv, 0.1, 1e-5, True), a.iters)
        res["apply_nobits_us"], res["apply_nobits_TBps"] = round(us, 1), round(2 * nb / us / 1e6, 2)
        y, sm, si = L.bn_fwd_part(x, part, None, g, b, rm, rv, 0.1, 1e-5, True)
        us = timeit(lambda: L.bn_bwd_part(r, x, part, g, sm, si, False, None, None), a.iters)
        res["dx_us"], res["dx_TBps"] = round(us, 1), round(3 * nb / us / 1e6, 2)
        out.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
