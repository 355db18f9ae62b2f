#!/usr/bin/env python3
"""Every kernel of ONE steady-state training step from a rocprofv3 --kernel-trace CSV, in launch order, with its
hardware queue, grid, duration and the time its queue idled before it -- to attribute step time to layers and to
see which stream a kernel ran on.  Aggregates per (kernel class, grid) too.

    python tools/step_calls.py gpurun_out/prof/run_kernel_trace.csv [--step 2] [--out f.md]
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
    ap.add_argument("--step", type=int, default=2, help="which softmax-xent-delimited step (0-based, after warmup)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "softmax_xent_kernel" in r["Kernel_Name"] or
             ("softmax_xent" in r["Kernel_Name"] and "bwd" not in r["Kernel_Name"])]
    if len(marks) < a.step + 2:
        sys.exit("not enough steps in the trace")
    lo, hi = marks[-(a.step + 2)], marks[-(a.step + 1)]
    step = rows[lo:hi]
    t0 = int(step[0]["Start_Timestamp"])
    qkey = "Queue_Id" if "Queue_Id" in step[0] else ("Stream_Id" if "Stream_Id" in step[0] else None)
    last_end = {}
    out = ["| # | start ms | queue | kernel | grid | us | queue idle before (us) |", "|---|---|---|---|---|---|---|"]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for i, r in enumerate(step):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get(qkey, "?") if qkey else "?"
        idle = (s - last_end[q]) / 1e3 if q in last_end else 0.0
        last_end[q] = e
        name = short(r["Kernel_Name"])
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        out.append("| %d | %.3f | %s | %s | %s | %.1f | %.1f |" % (i, (s - t0) / 1e6, q, name, grid, (e - s) / 1e3,
                                                                    idle))
        k = (name, grid, q)
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    span = (int(step[-1]["End_Timestamp"]) - t0) / 1e6
    out.append("\nstep span %.3f ms, %d kernels\n" % (span, len(step)))
    out.append("| kernel | grid | queue | calls | total us |")
    out.append("|---|---|---|---|---|")
    for (n, g, q), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append("| %s | %s | %s | %d | %.1f |" % (n, g, q, c, t))
    text = "\n".join(out)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
