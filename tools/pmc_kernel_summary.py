#!/usr/bin/env python3
"""Mean PMC counters of one kernel (name substring) over the rocprofv3 counter-collection CSVs under a directory, plus
the derived shares: MFMA-busy fraction of the SIMD cycles (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), and the wait /
VALU shares of the wave cycles.

    python tools/pmc_kernel_summary.py gpurun_out/linprof_28 lin_wgrad
"""
import collections
import csv
import glob
import os
import sys


def main():
    root, key = sys.argv[1], sys.argv[2]
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    v = {k: sum(x) / len(x) for k, x in vals.items()}
    for k in sorted(v):
        print("%-28s %.4g" % (k, v[k]))
    if "GRBM_GUI_ACTIVE" in v and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        print("MFMA busy        %.1f %%" % (100 * v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 1024)))
    if "SQ_WAVE_CYCLES" in v:
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY"):
            if c in v:
                print("%-16s %.1f %% of wave cycles" % (c, 100 * v[c] / v["SQ_WAVE_CYCLES"]))


if __name__ == "__main__":
    main()
