#!/usr/bin/env python3
"""The ResNet-50 stem forward conv (pixel-pair form, conv_fwd_c8 with the BN-statistics epilogue) at per-GPU batch
1024 under each LDS schedule (conv_set_stages(3, s): 1 single stage, 2 two-stage ring, 3 register-pipelined),
interleaved rounds, median us.

    python tools/stem_fwd_ab.py [--batch 1024]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops import conv as conv_ops  # noqa: E402
from dtg.ops._native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(a.batch, 3, 224, 224, generator=g).to(dev, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(dev, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    x8, w8, (rk, sk) = conv_ops.stem_pairs(x, w, 2, 3)
    times = {s: [] for s in (0, 1, 2, 3)}  # 0: the streaming kernel (gemm_expand.hip), 1-3: tiled schedules
    ref = None
    ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for sc in times:
            L.stem_stream_set(1 if sc == 0 else 0)
            L.conv_set_stages(3, max(sc, 1))
            y, part = L.conv_fwd_c8(x8, w8, rk, sk, 2, 0, True, stride_w=1)
            if ref is None:
                ref = y.float()
            assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-3, sc
            ev[0].record()
            for _ in range(5):
                L.conv_fwd_c8(x8, w8, rk, sk, 2, 0, True, stride_w=1)
            ev[1].record()
            torch.cuda.synchronize()
            times[sc].append(ev[0].elapsed_time(ev[1]) / 5 * 1e3)
    L.conv_set_stages(3, 0)
    L.stem_stream_set(1)
    print(json.dumps({("stream" if s == 0 else f"tiled_sched{s}"): round(sorted(v)[len(v) // 2], 1) for s, v in times.items()}), flush=True)


if __name__ == "__main__":
    main()
