#!/usr/bin/env python3
"""Practical HBM ceilings on this card for the streaming kernels' comparisons: write-only (fill), read+write
(copy) and read-only (sum) over a 1.64 GB bf16 tensor (ResNet-50's stage-1 activation at batch 1024)."""
import json

import torch


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    n = 3211264 * 256
    a = torch.empty(n, device="cuda", dtype=torch.bfloat16).normal_()
    b = torch.empty_like(a)
    nb = n * 2
    out = {"bytes": nb}
    out["fill_TBps"] = round(nb / timeit(lambda: b.fill_(1.0)) / 1e6, 2)
    out["copy_TBps"] = round(2 * nb / timeit(lambda: b.copy_(a)) / 1e6, 2)
    out["read_TBps"] = round(nb / timeit(lambda: a.sum(dtype=torch.float32)) / 1e6, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
