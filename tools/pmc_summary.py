#!/usr/bin/env python3
"""Summarise tools/pmc_ops.sh output: per case, the dtg kernel's counters averaged over dispatches,
plus derived ratios (wave-cycle split, HBM bytes, LDS conflict rate).

    python tools/pmc_summary.py gpurun_out/pmc [--out profiles/x/pmc.md]
"""
import collections
import csv
import glob
import os
import sys


def load(case_dir):
    """{kernel name: ({counter: mean over dispatches}, meta)} for the dtg kernels of one case."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(case_dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "dtg::" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"][:110]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"], "lds": r["LDS_Block_Size"],
                       "grid": r["Grid_Size"], "wg": r["Workgroup_Size"]}
    return {k: ({c: sum(v) / len(v) for c, v in d.items()}, meta[k]) for k, d in vals.items()}


def main():
    root = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    lines = []
    for case in sorted(os.listdir(root)):
      for kname, (c, m) in load(os.path.join(root, case)).items():
        lines.append(f"## {case}: {kname}\n{m}")
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        for k in sorted(c):
            lines.append(f"  {k:24s} {c[k]:16.0f}")
        lines.append(f"  wave-cycle split: active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}  "
                     f"wait(waitcnt/barrier) {c.get('SQ_WAIT_ANY', 0) / wc:.2f}  "
                     f"issue-stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}")
        if "FETCH_SIZE" in c:
            lines.append(f"  HBM read ~{2 * c['FETCH_SIZE'] / 1024:.1f} MB (2 x FETCH_SIZE), "
                         f"write {c.get('WRITE_SIZE', 0) / 1024:.1f} MB")
        if c.get("SQ_INSTS_LDS"):
            lines.append(f"  LDS bank-conflict cycles per LDS instr {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_INSTS_LDS']:.2f}")
    txt = "\n".join(lines)
    print(txt)
    if out:
        os.makedirs(os.path.dirname(out), exist_ok=True)
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
