#!/usr/bin/env python3
"""Express every kernel class of a whole-step PMC table (tools/pmc_step.py output, e.g.
profiles/r04_pmc_step/pmc_step_resnet.md) as a percentage of the HBM ceiling measured by dtg's own streaming
probe (tools/hbm_probe.py, csrc/kernels/stream_probe.hip).

The ceiling depends on the class's read/write mix: the probe's best rates are read-only, read-2/write-1, copy
and write-only; a class with write fraction f_w = W / (R + W) is compared against the piecewise-linear
interpolation between them (f_w = 0, 1/3, 1/2, 1).

    python tools/roof_pct.py profiles/r04_pmc_step/pmc_step_resnet.md profiles/r05_hbm_probe/hbm_probe.log
"""
import json
import sys


def ceilings(probe_log):
    summ = None
    for line in open(probe_log):
        if line.startswith('{"summary"'):
            summ = json.loads(line)["summary"]
    if summ is None:
        raise SystemExit("no summary line in %s" % probe_log)
    return [(0.0, summ["read"]), (1.0 / 3.0, summ["read2_write1"]), (0.5, summ["copy"]), (1.0, summ["write"])]


def ceiling_at(pts, fw):
    for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
        if fw <= x1:
            return y0 + (y1 - y0) * (fw - x0) / (x1 - x0)
    return pts[-1][1]


def main():
    table, probe = sys.argv[1], sys.argv[2]
    pts = ceilings(probe)
    rows = [l.rstrip("\n") for l in open(table) if l.startswith("|")]
    hdr = [c.strip() for c in rows[0].strip("|").split("|")]
    ir, iw, it, ims = (hdr.index("HBM read GB (x2)"), hdr.index("HBM write GB"), hdr.index("TB/s"),
                       next(i for i, h in enumerate(hdr) if h.startswith("GPU ms")))
    print("| kernel class | GPU ms | read GB | write GB | TB/s | write fraction | dtg HBM ceiling TB/s | % of ceiling |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows[2:]:
        c = [x.strip() for x in r.strip("|").split("|")]
        try:
            rd, wr, tb, ms = float(c[ir]), float(c[iw]), float(c[it]), float(c[ims])
        except ValueError:
            continue
        if rd + wr < 0.05:
            continue
        fw = wr / (rd + wr)
        ceil = ceiling_at(pts, fw)
        print("| %s | %.2f | %.1f | %.1f | %.2f | %.2f | %.2f | %d %% |" % (c[0], ms, rd, wr, tb, fw, ceil,
                                                                          round(100 * tb / ceil)))


if __name__ == "__main__":
    main()
