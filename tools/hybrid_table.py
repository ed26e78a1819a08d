"""Counter table of tools/hybrid_probe.sh: production wide kernel vs the hybrid row split.
usage: python tools/hybrid_table.py <dir>  (gpurun_out/<tag> of hybrid_probe.sh)
VALU issue share = SQ_INSTS_VALU x 2 cycles (the full-rate issue cost of a wave64 VALU
instruction on gfx950; v_perm / v_or_b32_sdwa take 4, so this is a lower bound) over the
SIMD cycles of the dispatch (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs); LDS busy =
SQ_LDS_IDX_ACTIVE over the CU cycles; clock = GRBM_GUI_ACTIVE / 8 / kernel time."""
import csv
import glob
import os
import re
import statistics
import sys
from collections import defaultdict


def load(d, kern):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def times(base, sh):
    out = {}
    for line in open(os.path.join(base, f"time_{sh}.log")):
        m = re.match(r"(prod dispatch|hybrid 8\+v)\s+([\d.]+)\s+[\d.]+\s+[\d.]+\s+([\d.]+)", line)
        if m:
            out["prod" if m.group(1).startswith("prod") else "hybrid"] = (float(m.group(2)), float(m.group(3)))
    return out


def main(base):
    print("shape,variant,pct_8TBs,kernel_us,lds_busy,valu_issue_share_min,valu_inst_per_wave,"
          "lds_inst_per_wave,clock_GHz")
    for sh in ("32_16", "20_16", "10_16", "10_12"):
        t = times(base, sh)
        for v, kern in (("prod", "rs_apply_lds"), ("hybrid", "hybrid_kernel")):
            c = {}
            for p in "AB":
                c.update(load(os.path.join(base, f"pmc_{v}_{sh}_{p}"), kern))
            if not c:
                continue
            g = c["GRBM_GUI_ACTIVE"] / 8  # cycles of one XCD
            w = c["SQ_WAVES"]
            lds = c["SQ_LDS_IDX_ACTIVE"] / (g * 256)
            valu = c["SQ_INSTS_VALU"] * 2 / (g * 256 * 4)
            us, pct = t.get(v, (float("nan"), float("nan")))
            clk = g / (us * 1e3) if us == us else float("nan")
            print(f"RS({sh.replace('_', ',')}),{v},{pct},{us},{lds:.3f},{valu:.3f},"
                  f"{c['SQ_INSTS_VALU'] / w:.0f},{c['SQ_INSTS_LDS'] / w:.0f},{clk:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
