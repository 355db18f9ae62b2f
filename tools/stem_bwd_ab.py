#!/usr/bin/env python3
"""The ResNet-50 stem's fused forward + backward at batch N (default 1024) with the backward's pass 2 fused into
the conv weight gradient (models/resnet_fused._STEM_FUSED_WG = 1) or not (0), interleaved; HIP-event time of the
backward alone.

    python tools/stem_bwd_ab.py [--batch 1024] [--rounds 3] [--only 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.models import resnet_fused  # noqa: E402
from dtg.models.layers import ConvBN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", type=int, default=-1, help="time only this setting (profiling)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    x = torch.randn(a.batch, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    torch.manual_seed(0)
    stem = ConvBN(3, 64, 7, 2, 3).to(dev)
    stem.conv.weight.data = stem.conv.weight.data.to(torch.bfloat16)
    stem.train()
    y = resnet_fused.stem_pool(stem, x)
    gy = torch.randn_like(y)

    def bwd(fused):
        resnet_fused._STEM_FUSED_WG = bool(fused)
        yy = resnet_fused.stem_pool(stem, x)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        yy.backward(gy)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3

    settings = [a.only] if a.only >= 0 else [1, 0]
    for r in range(a.rounds):
        out = []
        for f in settings:
            ts = sorted(bwd(f) for _ in range(5))
            out.append("fused=%d %.1f us" % (f, ts[2]))
        print("round %d: %s" % (r, "  ".join(out)), flush=True)


if __name__ == "__main__":
    main()
