"""Table of PMC counters per shape from a tools/pmc_shapes.sh output dir (the hot
kernel's dispatches only, median per counter), with derived ratios."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def load(d, kernel="rs_apply"):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc_counter_collection.csv")) + glob.glob(os.path.join(d, "*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def main(src):
    shapes = sorted({os.path.basename(p).split("_")[1:3].__str__() for p in []})
    rows = []
    for log in sorted(glob.glob(os.path.join(src, "kbench_*.log"))):
        k, m = os.path.basename(log)[7:-4].split("_")
        c = {}
        for p in "AB":
            c.update(load(os.path.join(src, f"pmc_{k}_{m}_{p}")))
        pct = None
        for line in open(log):
            if line.startswith("prod dispatch"):
                pct = float(line.split()[-1])
        rows.append((int(k), int(m), pct, c))
    keys = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
            "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
            "GRBM_GUI_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"]
    print("k,m,%8TB/s," + ",".join(keys) + ",lds_busy,valu_busy,conflict_frac,valu_per_wave,lds_per_wave")
    for k, m, pct, c in sorted(rows):
        g = c.get("GRBM_GUI_ACTIVE", 0) or 1
        busy = c.get("SQ_BUSY_CYCLES", 0) or 1
        # SQ_LDS_IDX_ACTIVE: LDS-array cycles summed over CUs; GRBM_GUI_ACTIVE: GPU clocks
        # summed over the 8 XCDs (MI355X_MICROARCH.md) -> per-CU LDS utilisation
        lds_busy = c.get("SQ_LDS_IDX_ACTIVE", 0) / (g / 8 * 256)
        valu_busy = c.get("SQ_ACTIVE_INST_VALU", 0) / (g / 8 * 256 * 4)
        cf = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 1))
        w = c.get("SQ_WAVES", 1) or 1
        print(f"{k},{m},{pct}," + ",".join(f"{c.get(x, float('nan')):.4g}" for x in keys) +
              f",{lds_busy:.3f},{valu_busy:.3f},{cf:.3f},{c.get('SQ_INSTS_VALU', 0) / w:.0f},"
              f"{c.get('SQ_INSTS_LDS', 0) / w:.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
