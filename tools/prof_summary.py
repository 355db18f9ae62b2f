#!/usr/bin/env python3
"""Steady-state per-step kernel breakdown from a rocprofv3 --kernel-trace run of bench.py.

Warmup dispatches (MIOpen find, first-touch allocations) are dropped by keeping only the kernels
after the (skip+1)-th softmax-xent launch (one per training step), so the table is per timed step.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv [--skip 4] [--top 40] [--out f.md]
    python tools/prof_summary.py gpurun_out/prof/run_results.db          (rocprofv3's default output)
"""
import argparse
import collections
import csv
import re


def _targs(name, start):
    """Top-level template arguments of the template whose '<' is at name[start]."""
    args, depth, cur = [], 0, ""
    for ch in name[start + 1:]:
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            if depth == 0:
                args.append(cur.strip())
                return args
            depth -= 1
        if ch == "," and depth == 0:
            args.append(cur.strip())
            cur = ""
        else:
            cur += ch
    return args


def short(name):
    m = (re.search(r"dtg::(?:\(anonymous namespace\)::)?(\w+?)_kernel", name)
         or re.search(r"dtg::(?:\(anonymous namespace\)::)?(\w+)", name))
    if m:
        base = m.group(1)
        if base == "gemm" and "gemm_kernel<" in name:
            # gemm_kernel<Cfg, AKC, BKC, SA, SB, BNMODE, FAST, BNPF>: the BN-epilogue mode tells the classes apart
            a = _targs(name, name.index("gemm_kernel<") + len("gemm_kernel"))
            if len(a) > 5 and a[5].isdigit() and a[5] != "0":
                base += f" bn{a[5]}"
        return base
    return name[:48]


def load(path):
    """Kernel rows from a rocprofv3 kernel-trace CSV or its default rocpd SQLite output (.db)."""
    if not path.endswith(".db"):
        return list(csv.DictReader(open(path)))
    import sqlite3
    con = sqlite3.connect(path)
    return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
            for n, s, e in con.execute("select name, start, end from kernels")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=4, help="warmup steps to drop")
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = sorted(load(a.trace), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "softmax_xent_kernel" in r["Kernel_Name"]]  # forward: one per step
    if len(marks) <= a.skip + 1:
        raise SystemExit(f"only {len(marks)} steps in the trace")
    lo, hi = marks[a.skip], marks[-1]
    steps = len(marks) - 1 - a.skip
    seg = rows[lo + 1:hi + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values()) / steps  # sum of kernel durations: exceeds wall with concurrent streams
    # union of the kernels' [start, end) intervals: the time at least one kernel was running
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
    union, cur_s, cur_e = 0, iv[0][0], iv[0][1]
    for s0, e0 in iv[1:]:
        if s0 > cur_e:
            union += cur_e - cur_s
            cur_s, cur_e = s0, e0
        else:
            cur_e = max(cur_e, e0)
    union = (union + cur_e - cur_s) / 1e3 / steps
    wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3 / steps
    lines = [f"steady-state step: wall {wall / 1e3:.2f} ms, GPU-busy (interval union) {union / 1e3:.2f} ms, "
             f"sum of kernel times {busy / 1e3:.2f} ms over {steps} steps",
             f"{'kernel':44s} {'calls/step':>10s} {'ms/step':>8s} {'%sum':>5s}"]
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        lines.append(f"{k:44s} {n / steps:10.1f} {us / steps / 1e3:8.3f} {100 * us / steps / busy:5.1f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
