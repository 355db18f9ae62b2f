#!/usr/bin/env python3
"""PMC comparison of dtg's production GEMM and hipBLASLt on one BERT shape, for rocprofv3 --pmc passes.

    run:      rocprofv3 --pmc <counters> -d <dir> -o run --output-format csv -- \\
                  python3 tools/gemm_pmc_lib.py run <case>
    summary:  python3 tools/gemm_pmc_lib.py summary <dir> [<dir> ...] [--out file.md]

Cases (32768 tokens, BERT-base): ffn1 = x W1^T + b1 with GELU and GELU'(pre) saved (dtg) / torch addmm + gelu
(hipBLASLt epilogue GELU, no GELU'); ffn2 = f1 W2^T + b2 (dtg bias epilogue / torch addmm).  ITERS launches each.
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(case):
    import torch
    import dtg  # noqa: F401
    from dtg.ops._native import lib
    L = lib()
    dev = torch.device("cuda")
    iters = int(os.environ.get("ITERS", "10"))
    M, N, K = (32768, 3072, 768) if case == "ffn1" else (32768, 768, 3072)
    g = torch.Generator(device="cpu").manual_seed(0)
    A = (torch.rand(M, K, generator=g) * 2 - 1).to(dev, torch.bfloat16)
    B = (torch.rand(N, K, generator=g) * 0.1 - 0.05).to(dev, torch.bfloat16)
    bias = torch.rand(N, generator=g).to(dev) * 0.1
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    aux = torch.empty_like(out)
    if case == "ffn1":
        ours = lambda: L.gemm(A, True, B, True, out, 1.0, 0.0, bias, 2, 0, aux, 3)  # noqa: E731
        theirs = lambda: torch._addmm_activation(bias.bfloat16(), A, B.t(), use_gelu=True)  # noqa: E731
    else:
        ours = lambda: L.gemm(A, True, B, True, out, 1.0, 0.0, bias, 0, 0)  # noqa: E731
        theirs = lambda: torch.addmm(bias.bfloat16(), A, B.t(), out=out)  # noqa: E731
    for fn in (ours, theirs):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()


def summary(dirs, out=None):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"]
                who = "dtg" if "dtg::" in n else ("hipBLASLt" if "Cijk_" in n else None)
                if who is None:
                    continue
                key = (os.path.basename(os.path.normpath(d)).split("_")[0], who, n[:60])
                vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = ["| case | kernel | name | us (GRBM / 8 XCDs at 2.4 GHz) | MFMA busy % | wave-cycles (M) | SQ_WAIT_INST_ANY / "
             "wave-cycles | LDS instr (M) | LDS bank conflict cycles / LDS instr | L2 hit % |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for (case, who, name), d in sorted(vals.items()):
        m = {c: sum(v) / len(v) for c, v in d.items()}
        gui = m.get("GRBM_GUI_ACTIVE")
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES")
        # SQ_VALU_MFMA_BUSY_CYCLES counts per SIMD-cycle summed over the chip: 256 CUs x 4 SIMDs
        mf = "%.1f" % (100.0 * busy / (gui / 8 * 1024)) if gui and busy else "-"
        wait = m.get("SQ_WAIT_INST_ANY"), m.get("SQ_WAVE_CYCLES")
        wt = "%.2f" % (wait[0] / wait[1]) if all(wait) else "-"
        lds = m.get("SQ_LDS_BANK_CONFLICT"), m.get("SQ_INSTS_LDS")
        lc = "%.2f" % (lds[0] / lds[1]) if all(lds) else "-"
        hit = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
        hr = "%.1f" % (100.0 * hit[0] / (hit[0] + hit[1])) if all(v is not None for v in hit) and sum(hit) else "-"
        us = "%.1f" % (gui / 8 / 2400.0) if gui else "-"
        wc = "%.1f" % (wait[1] / 1e6) if wait[1] else "-"
        li = "%.2f" % (lds[1] / 1e6) if lds[1] is not None else "-"
        lc = "%.2f" % (lds[0] / lds[1]) if lds[0] is not None and lds[1] else "-"
        lines.append(f"| {case} | {who} | `{name[:44]}` | {us} | {mf} | {wc} | {wt} | {li} | {lc} | {hr} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        args = sys.argv[2:]
        out = None
        if "--out" in args:
            i = args.index("--out")
            out = args[i + 1]
            args = args[:i] + args[i + 2:]
        summary(args, out)
