#!/usr/bin/env python3
"""In-process A/B of the conv output tiles (conv_force_tile, csrc/kernels/conv.hip) on the ResNet-50 stride-1
3x3 layers at per-GPU batch 1024: forward with BN statistics and data gradient with the BN-backward epilogue;
--strided: the stride-2 forwards instead (the first 3x3 of stages 2-4 and the 1x1 projections).
Tile codes: 0 heuristic (128x128 / 256x64, 4 waves), 1 128x256 8-wave RP, 2 256x128 8-wave RP, 3 128x256 8-wave
single stage.  Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); every forced tile's
output is checked against the heuristic's.

    python tools/conv_tile_ab.py [--batch 1024] [--codes 0,1,2,3] [--rounds 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402

LAYERS = [(56, 64), (28, 128), (14, 256), (7, 512)]  # (H, C = K) of the stride-1 3x3 convs


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--codes", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--strided", action="store_true")
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    codes = [int(c) for c in a.codes.split(",")]
    g = torch.Generator(device="cpu").manual_seed(0)
    layers = ([(H, C, C, 3) for H, C in [(56, 128), (28, 256), (14, 512)]] +
              [(H, C, 2 * C, 1) for H, C in [(56, 256), (28, 512), (14, 1024)]]) if a.strided else \
        [(H, C, C, 3) for H, C in LAYERS]
    for H, C, K, R in layers:
        N = a.batch
        s_ = 2 if a.strided else 1
        x = (torch.rand(N, H, H, C, generator=g) * 2 - 1).to(dev, torch.bfloat16)
        w = ((torch.rand(K, R, R, C, generator=g) * 2 - 1) / (R * C ** 0.5)).to(dev, torch.bfloat16)
        dy = (torch.rand(N, H, H, C, generator=g) * 2 - 1).to(dev, torch.bfloat16)
        ch = [(torch.rand(C, generator=g) + 0.5).to(dev) for _ in range(4)]
        ops = {"fwd_bn": (0, lambda: L.conv_fwd_bn(x, w, s_, R // 2))}
        if not a.strided:
            ops["dgrad_bn"] = (1, lambda: L.conv_dgrad_bn(dy, w, H, H, 1, 1, x.view(-1, C), *ch))
        flops = 2.0 * N * (H // s_) ** 2 * K * R * R * C
        for name, (which, fn) in ops.items():
            ref = None
            res = {c: [] for c in codes}
            errs = {}
            for r in range(a.rounds):
                for c in codes:
                    L.conv_force_tile(which, c)
                    fn()
                    if r == 0:
                        out = fn()[0].float()
                        torch.cuda.synchronize()
                        if c == codes[0]:
                            ref = out
                        else:
                            errs[c] = ((out - ref).norm() / ref.norm()).item()
                    res[c].append(timed(fn, a.iters))
                L.conv_force_tile(which, 0)
            line = {"layer": f"{H}x{H}x{C}->{K} {R}x{R}/s{s_}", "op": name}
            for c in codes:
                t = sorted(res[c])[len(res[c]) // 2]
                line[str(c)] = {"us": round(t, 1), "tflops": round(flops / t / 1e6, 1)}
                if c in errs:
                    line[str(c)]["rel_err_vs_0"] = errs[c]
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
