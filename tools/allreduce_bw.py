#!/usr/bin/env python3
"""All-reduce bus bandwidth versus message size (SURVEY §7.3 phase 4: "bus bandwidth versus size at
2/4/8 GPUs"), one process per GPU over RCCL (xGMI), or gloo on the CPU.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/allreduce_bw.py \
        [--min_kb 64] [--max_mb 256] [--dtype bf16] [--iters 20] [--json out.jsonl]

Per size: mean time of one in-place all_reduce(SUM) (max over ranks), algorithm bandwidth = bytes/t
and bus bandwidth = algbw * 2(n-1)/n (the ring-equivalent per-link rate; on a fully connected
8-GPU xGMI node it can exceed one link's ~153 GB/s because RCCL spreads channels over all 7 peers).
Also times the gradient buckets DataParallel would launch for ResNet-50 (``--bucket_mb``), the
communication a training step overlaps with backward.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min_kb", type=float, default=64)
    ap.add_argument("--max_mb", type=float, default=256)
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp32"))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from dtg.parallel import comm

    rank, _, world, device = comm.init()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    esz = 2 if dt == torch.bfloat16 else 4
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    rows = []

    def measure(nbytes, tag):
        n = max(1, int(nbytes) // esz)
        t = torch.ones(n, dtype=dt, device=device)
        for _ in range(a.warmup):
            dist.all_reduce(t) if world > 1 else None
        sync()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            if world > 1:
                dist.all_reduce(t)
        sync()
        dt_s = comm.all_reduce_max((time.perf_counter() - t0) / a.iters, device)
        alg = n * esz / dt_s / 1e9 if dt_s > 0 else 0.0
        row = {"tag": tag, "bytes": n * esz, "n_ranks": world, "us": dt_s * 1e6, "algbw_GBs": alg,
               "busbw_GBs": alg * 2 * (world - 1) / world if world > 1 else 0.0, "dtype": a.dtype}
        rows.append(row)
        if rank == 0:
            print(json.dumps(row), flush=True)

    size = a.min_kb * 1024
    while size <= a.max_mb * 1024 * 1024:
        measure(size, "sweep")
        size *= 2
    # ResNet-50's gradient (25.6 M parameters) in DataParallel-sized buckets
    total = 25_557_032 * esz
    b = int(a.bucket_mb * 1024 * 1024)
    while total > 0:
        measure(min(b, total), f"resnet50_bucket_{a.bucket_mb:g}MB")
        total -= b
    if rank == 0 and a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    comm.shutdown()


if __name__ == "__main__":
    main()
