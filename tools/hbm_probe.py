#!/usr/bin/env python3
"""HBM ceiling of this card, measured with dtg's own streaming kernels (csrc/kernels/stream_probe.hip).

Replaces tools/hbm_roof.py (torch copy_ / sum, which read *below* what dtg's BN passes sustain): read-only,
write-only, copy and read-2/write-1 over 1.64 GB buffers (ResNet-50's stage-1 activation at batch 1024, far
past the 256 MiB Infinity Cache), 16-B vector accesses, 1/2/4/8 vectors in flight per lane, plain and
non-temporal, grids of 1-8 workgroups per CU.  Prints one JSON line per variant and a summary line with the
best rate per kind -- the ceilings tools/pmc_step.py expresses the ResNet step's kernel classes against.

    python tools/hbm_probe.py [--mb 1640] [--iters 10] [--quick]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KINDS = {0: "read", 1: "write", 2: "copy", 3: "read2_write1"}
# bytes moved per 16-B vector of the buffer size
TRAFFIC = {0: 1, 1: 1, 2: 2, 3: 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1640)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--quick", action="store_true", help="only the 4-in-flight, 1024-workgroup variants")
    args = ap.parse_args()
    import dtg  # noqa: F401
    from dtg.ops import lib
    L = lib()
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nbytes = args.mb * 2 ** 20 // 16 * 16
    a = torch.randint(0, 2 ** 30, (nbytes // 4,), device=dev, dtype=torch.int32)
    b = torch.randint(0, 2 ** 30, (nbytes // 4,), device=dev, dtype=torch.int32)
    o = torch.empty_like(a)
    sink = torch.zeros(8 * cus, device=dev, dtype=torch.int32)
    grids = [cus * k for k in ((4,) if args.quick else (1, 2, 4, 8))]
    unrolls = (4,) if args.quick else (1, 2, 4, 8)
    best = {}
    for kind in KINDS:
        for nt in (False, True):
            for u in unrolls:
                for g in grids:
                    fn = lambda: L.stream_probe(kind, a, b, o, sink, g, u, nt)
                    fn()
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(args.iters):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    us = s.elapsed_time(e) / args.iters * 1e3
                    tbps = TRAFFIC[kind] * nbytes / us / 1e6
                    rec = {"kind": KINDS[kind], "nt": nt, "in_flight": u, "wgs": g, "us": round(us, 1),
                           "TBps": round(tbps, 3)}
                    print(json.dumps(rec), flush=True)
                    if tbps > best.get(KINDS[kind], {"TBps": 0})["TBps"]:
                        best[KINDS[kind]] = rec
    # correctness of the copy / add forms (the probe is a measurement, but a wrong kernel measures nothing)
    L.stream_probe(2, a, None, o, sink, grids[0], 4, False)
    assert torch.equal(o, a), "copy probe wrote wrong data"
    L.stream_probe(3, a, b, o, sink, grids[0], 4, True)
    assert torch.equal(o, a + b), "read2/write1 probe wrote wrong data"
    print(json.dumps({"summary": {k: v["TBps"] for k, v in best.items()}, "best": best, "bytes": nbytes,
                      "cus": cus}))


if __name__ == "__main__":
    main()
