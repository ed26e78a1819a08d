"""Table of tools/jobs.sh pmc_forms: per kernel form, % of 8 TB/s (trace), LDS-array busy, VALU
issue share, waves resident per SIMD, wait share and clock.
usage: python tools/pmc_forms_table.py <gpurun_out/tag> <bytes per launch> <order> [...]
LDS busy = SQ_LDS_IDX_ACTIVE / CU cycles; VALU share = SQ_ACTIVE_INST_VALU (quad-cycles x 4)
/ SIMD cycles; waves/SIMD = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / 4 (both in quad-cycles per SE
sum, a ratio); wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES; clock = GRBM_GUI_ACTIVE / 8 / time."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def counters(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "rs_apply_lds" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def kernel_us(d):
    ds = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "rs_apply_lds" in r["Kernel_Name"]:
                ds.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ds = ds[len(ds) // 3:]  # drop the warm-up third
    return statistics.mean(ds) if ds else float("nan")


def main(base, nbytes, orders):
    print("form,pct_8TBs,kernel_us,lds_busy,valu_share,waves_per_simd,wait_share,valu_inst_per_wave,"
          "lds_inst_per_wave,bank_conflict_share,clock_GHz")
    for o in orders:
        c = {}
        for p in "AB":
            c.update(counters(os.path.join(base, f"pmc_{o}_{p}")))
        us = kernel_us(os.path.join(base, f"trace_{o}"))
        if not c:
            continue
        g = c["GRBM_GUI_ACTIVE"] / 8
        cu = g * 256
        w = c["SQ_WAVES"]
        print(f"{o},{nbytes / (us * 1e-6) / 8e12 * 100:.2f},{us:.1f},"
              f"{c['SQ_LDS_IDX_ACTIVE'] / cu:.3f},{c['SQ_ACTIVE_INST_VALU'] * 4 / (cu * 4):.3f},"
              f"{c['SQ_WAVE_CYCLES'] / c['SQ_BUSY_CYCLES'] / 4:.2f},"
              f"{c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f},{c['SQ_INSTS_VALU'] / w:.0f},"
              f"{c['SQ_INSTS_LDS'] / w:.0f},{c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.3f},"
              f"{g / (us * 1e3):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3:])
