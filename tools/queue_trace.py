#!/usr/bin/env python3
"""Hardware-queue view of a rocprofv3 --kernel-trace run: which queue every dispatch went to, and whether
the collective (RCCL or the DTG_COMM_EMULATE spin kernel) ran concurrently with the weight-gradient side
stream or serialised against it.

    python tools/queue_trace.py gpurun_out/qt/<pid>_kernel_trace.csv [--skip 4] [--out profiles/.../queues.md]

Per steady-state step (kernels between the (skip+1)-th and last softmax-xent launch, one per step):

* per Queue_Id (and Stream_Id): dispatches, busy ms, the three largest kernel classes;
* for the collective queue(s): how much of the collective time overlapped kernels on OTHER queues, and how
  many side-stream kernels STARTED while a collective was running (zero would mean the side stream sat
  behind the collective: a shared queue or a cross-stream wait);
* the tail: time from the last non-collective kernel of the step to the end of the last collective
  (communication left exposed after backward), and from that to the next step's first kernel.
"""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def is_comm(name):
    """Collective-side dispatches: RCCL kernels, dtg's emulated collective (comm_spin / comm_emu), and -- under
    DTG_COMM_QUEUE_PROBE=1 -- the one-rank all-gather's copy on the process group's stream (a ROCclr blit)."""
    n = name.lower()
    return ("comm_spin" in n or "comm_emu" in n or "nccl" in n or "rccl" in n or "copybuffer" in n
            or "rocclr" in n)


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def overlap(a, b):
    """Total length of (union of a) intersected with (union of b)."""
    return union(a) + union(b) - union(a + b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=4)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    marks = [i for i, r in enumerate(rows) if "softmax_xent_kernel" in r["Kernel_Name"]]
    if len(marks) <= a.skip + 1:
        raise SystemExit(f"only {len(marks)} steps in the trace")
    steps = len(marks) - 1 - a.skip
    seg = rows[marks[a.skip]:marks[-1]]
    qkey = lambda r: (r.get("Queue_Id", "?"), r.get("Stream_Id", "?"))  # noqa: E731
    byq = collections.defaultdict(list)
    for r in seg:
        byq[qkey(r)].append(r)
    out = [f"steady state: {steps} steps, {len(seg)} dispatches\n",
           "| queue | stream | dispatches/step | busy ms/step | top kernels (ms/step) |", "|---|---|---|---|---|"]
    comm_q = set()
    for k, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        cls = collections.Counter()
        for r in rs:
            cls[short(r["Kernel_Name"])] += (r["e"] - r["s"]) / 1e6 / steps
        busy = union([(r["s"], r["e"]) for r in rs]) / 1e6 / steps
        top = ", ".join(f"{n} {t:.2f}" for n, t in cls.most_common(3))
        out.append(f"| {k[0]} | {k[1]} | {len(rs) / steps:.1f} | {busy:.2f} | {top} |")
        if any(is_comm(r["Kernel_Name"]) for r in rs):
            comm_q.add(k)
    comm = [r for r in seg if is_comm(r["Kernel_Name"])]
    if comm:
        civ = [(r["s"], r["e"]) for r in comm]
        other = [(r["s"], r["e"]) for r in seg if not is_comm(r["Kernel_Name"])]
        ct = union(civ)
        ov = overlap(civ, other)
        out.append("")
        out.append(f"collective kernels: {len(comm) / steps:.1f}/step on queue(s) {sorted(q[0] for q in comm_q)}, "
                   f"{ct / 1e6 / steps:.3f} ms/step; overlapped with other queues' kernels: {ov / max(ct, 1) * 100:.1f} %")
        for k, rs in byq.items():
            if k in comm_q:
                continue
            starts = sum(1 for r in rs if any(s <= r["s"] < e for s, e in civ))
            out.append(f"  queue {k[0]} stream {k[1]}: {starts / steps:.1f} dispatches/step started while a "
                       f"collective was running")
        # tail per step: from the last compute kernel before each step boundary to the last collective end
        tails = []
        for i in range(a.skip, len(marks) - 1):
            st_rows = rows[marks[i]:marks[i + 1]]
            last_comm = max((r["e"] for r in st_rows if is_comm(r["Kernel_Name"])), default=None)
            apply = [r for r in st_rows if "apply" in r["Kernel_Name"]]
            if last_comm is None or not apply:
                continue
            pre = [r["e"] for r in st_rows if not is_comm(r["Kernel_Name"]) and r["s"] < apply[0]["s"]]
            if pre:
                tails.append((last_comm - max(pre)) / 1e6)
        if tails:
            out.append(f"exposed collective tail (last collective end - last backward kernel end, before the "
                       f"optimizer apply): mean {sum(tails) / len(tails):.3f} ms, max {max(tails):.3f} ms")
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
