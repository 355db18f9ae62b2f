#!/usr/bin/env python3
"""Whole-step hardware counters per kernel class from rocprofv3 --pmc runs of bench.py (tools/pmc_step.sh):
MFMA busy share and HBM traffic of every kernel class in one training step.

    python tools/pmc_step.py gpurun_out/pmc_step [--steps 1] [--out profiles/x/pmc_step.md]

Normalisation (MI355X_MICROARCH.md): GRBM_GUI_ACTIVE is summed over the 8 XCDs, so a dispatch's cycles are
GRBM_GUI_ACTIVE / 8; SQ_VALU_MFMA_BUSY_CYCLES is summed over the SIMDs, so MFMA busy = it / (cycles * 1024
SIMDs).  FETCH_SIZE reads half of a wide coalesced streaming read's bytes on gfx950 and is doubled here
(the upper bound; narrow reads are counted once); FETCH_SIZE / WRITE_SIZE are in KiB.
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def load(d):
    """[(dispatch id, kernel, {counter: value})] in dispatch order"""
    rows = collections.OrderedDict()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = int(r["Dispatch_Id"])
            e = rows.setdefault(key, [r["Kernel_Name"], {}])
            e[1][r["Counter_Name"]] = e[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(k, v[0], v[1]) for k, v in sorted(rows.items())]


def last_steps(disp, steps):
    """the dispatches after the (steps+1)-th last softmax-xent forward (one per training step)"""
    marks = [i for i, (_, n, _) in enumerate(disp) if "softmax_xent" in n and "bwd" not in n]
    if len(marks) <= steps:
        return disp
    return disp[marks[-steps - 1] + 1:marks[-1] + 1] if steps else disp


def main():
    root = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 1
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    passes = sorted(glob.glob(os.path.join(root, "p*")))
    for ip, p in enumerate(passes):
        for _, name, c in last_steps(load(p), steps):
            k = short(name)
            for cn, v in c.items():
                if cn == "GRBM_GUI_ACTIVE":  # in every pass: the mean over passes
                    v /= len(passes)
                agg[k][cn] += v
            if ip == 0:
                calls[k] += 1
    lines = ["| kernel class | calls/step | GPU ms/step (GRBM/8 at 2.4 GHz) | MFMA busy | HBM read GB (x2) | HBM write GB | TB/s |",
             "|---|---|---|---|---|---|---|"]
    tot = collections.defaultdict(float)
    for k in sorted(agg, key=lambda k: -agg[k].get("GRBM_GUI_ACTIVE", 0)):
        c = agg[k]
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc <= 0:
            continue
        ms = cyc / 2.4e9 * 1e3 / steps
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (cyc * 1024)
        rd = 2 * c.get("FETCH_SIZE", 0) * 1024 / 1e9 / steps
        wr = c.get("WRITE_SIZE", 0) * 1024 / 1e9 / steps
        for n, v in (("ms", ms), ("mfma", c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)), ("cyc", cyc), ("rd", rd), ("wr", wr)):
            tot[n] += v
        lines.append(f"| {k} | {calls[k] / steps:.0f} | {ms:.2f} | {mf:.1%} | {rd:.1f} | {wr:.1f} | "
                     f"{(rd + wr) / ms if ms else 0:.2f} |")
    lines.append(f"| **all** | | {tot['ms']:.2f} | {tot['mfma'] / (tot['cyc'] * 1024):.1%} | {tot['rd']:.1f} | "
                 f"{tot['wr']:.1f} | {(tot['rd'] + tot['wr']) / tot['ms'] if tot['ms'] else 0:.2f} |")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
