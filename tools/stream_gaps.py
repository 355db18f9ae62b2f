#!/usr/bin/env python3
"""Where the main stream waits in a training step: idle gaps of each hardware queue inside the steady-state
step, and which kernels on the OTHER queues were running during them (the work the waiting queue was blocked
behind -- e.g. a main stream that waits for the side stream's weight gradients at a join).

    python tools/stream_gaps.py gpurun_out/qt/<pid>_kernel_trace.csv [--skip 4] [--min-us 5] [--out f.md]

Only gaps of at least --min-us count (shorter ones are dispatch latency).  For every queue: total gap time
per step and the kernel classes on other queues that overlapped its gaps (ms/step of overlap).
"""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=4)
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["q"] = r.get("Queue_Id", "?")
        r["k"] = short(r["Kernel_Name"])
    rows.sort(key=lambda r: r["s"])
    marks = [i for i, r in enumerate(rows) if "softmax_xent_kernel" in r["Kernel_Name"]]
    if len(marks) <= a.skip + 1:
        raise SystemExit(f"only {len(marks)} steps in the trace")
    steps = len(marks) - 1 - a.skip
    seg = rows[marks[a.skip]:marks[-1]]
    t0, t1 = seg[0]["s"], max(r["e"] for r in seg)
    byq = collections.defaultdict(list)
    for r in seg:
        byq[r["q"]].append(r)
    out = [f"steady state: {steps} steps, wall {(t1 - t0) / 1e6 / steps:.2f} ms/step; gaps >= {a.min_us} us\n"]
    for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        gaps, end = [], rs[0]["e"]
        for r in rs[1:]:
            if r["s"] - end >= a.min_us * 1e3:
                gaps.append((end, r["s"]))
            end = max(end, r["e"])
        gap_ms = sum(e - s for s, e in gaps) / 1e6 / steps
        cls = collections.Counter()
        others = [r for r in seg if r["q"] != q]
        j = 0
        for gs, ge in gaps:
            while j < len(others) and others[j]["e"] < gs - 10**7:
                j += 1
            for r in others[j:]:
                if r["s"] >= ge:
                    break
                ov = min(ge, r["e"]) - max(gs, r["s"])
                if ov > 0:
                    cls[r["k"]] += ov / 1e6 / steps
        out.append(f"queue {q}: {len(rs) / steps:.0f} dispatches/step, {len(gaps) / steps:.1f} gaps/step, "
                   f"{gap_ms:.3f} ms/step idle inside the step")
        for k, ms in cls.most_common(a.top):
            out.append(f"    {k:44s} {ms:7.3f} ms/step running on another queue during the gaps")
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
