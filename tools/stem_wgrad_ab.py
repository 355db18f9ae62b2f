"""Isolated timing of the stem conv's weight gradient (pixel-pair form, ops/conv.py stem_pairs) at ResNet-50's
stem shape under different LDS schedules (conv_set_stages(2, s)) and split-K workgroup targets.
python tools/stem_wgrad_ab.py [--batch 1024] [--iters 10]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    N = a.batch
    xp = torch.randn(N, 230, 115, 8, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, 112, 112, 64, device=dev).to(torch.bfloat16)
    ref = None
    for stages in (1, 2, 3):
        for wgs in (0, 512, 2048):
            L.conv_set_stages(2, stages)
            dw = torch.empty(64, 7, 4, 8, device=dev)
            fn = lambda: L.conv_wgrad(dy, xp, dw, 0.0, 2, 0, stride_w=1, target_wgs=wgs)  # noqa: E731
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = dw.clone()
            err = ((dw - ref).norm() / ref.norm()).item()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            print(f"stages={stages} target_wgs={wgs or 'default'}: {s.elapsed_time(e) / a.iters * 1e3:.1f} us "
                  f"(rel diff vs first {err:.1e})", flush=True)
    L.conv_set_stages(2, 0)


if __name__ == "__main__":
    main()
