"""Table of tools/jobs.sh pmc_bs: per kernel form of one shape, % of 8 TB/s (kernel trace), clock,
VALU instructions per input byte, VALU issue share, LDS issue share, waves per SIMD, wait
share and instruction-cache misses (development tool).
usage: python tools/pmc_bs_table.py <gpurun_out/tag> <k> <m> <S> <stripes> <form> [...]
VALU share = SQ_ACTIVE_INST_VALU x 4 / SIMD cycles (the counter is in quad-cycles, summed over
the chip); waves / SIMD = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / 4; wait share = SQ_WAIT_ANY /
SQ_WAVE_CYCLES; clock = GRBM_GUI_ACTIVE / 8 / kernel time (MI355X_MICROARCH.md "DVFS")."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

KERNELS = ("rs_bs", "rs_apply_lds", "rs_apply_vec")


def counters(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in KERNELS):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def kernel(d):
    ds, name, vgpr = [], "", 0
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in KERNELS):
                ds.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                name, vgpr = r["Kernel_Name"], int(r.get("VGPR_Count", 0) or 0)
    ds = ds[len(ds) // 3:]  # drop the warm-up third
    return (statistics.mean(ds) if ds else float("nan")), name, vgpr


def main(base, k, m, S, B, forms):
    nbytes = B * S * (k + m)
    inbytes = B * S * k
    print("form,kernel,vgprs,pct_8TBs,kernel_us,clock_GHz,valu_per_input_byte,valu_share,"
          "lds_share,waves_per_simd,wait_share,valu_inst_per_wave,vmem_inst_per_wave,"
          "icache_miss_per_wave,icache_miss_share")
    for o in forms:
        c = {}
        for p in "ABC":
            c.update(counters(os.path.join(base, f"pmc_{o}_{p}")))
        us, name, vgpr = kernel(os.path.join(base, f"trace_{o}"))
        if not c:
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        simd = cyc * 256 * 4
        w = c["SQ_WAVES"]
        vmem = c.get("SQ_INSTS_VMEM_RD", 0) + c.get("SQ_INSTS_VMEM_WR", 0)
        miss = c.get("SQC_ICACHE_MISSES", float("nan"))
        req = c.get("SQC_ICACHE_REQ", c.get("SQC_ICACHE_HITS", 0) + miss)
        short = "rs_bs (bit-sliced)" if "rs_bs" in name else ("rs_apply_lds" if "lds" in name else name[:20])
        print(f"{o},{short},{vgpr},{nbytes / (us * 1e-6) / 8e12 * 100:.2f},{us:.1f},{cyc / (us * 1e3):.2f},"
              f"{c['SQ_INSTS_VALU'] * 64 / inbytes:.2f},{c['SQ_ACTIVE_INST_VALU'] * 4 / simd:.3f},"
              f"{c.get('SQ_ACTIVE_INST_LDS', 0) * 4 / simd:.3f},"
              f"{c['SQ_WAVE_CYCLES'] / c['SQ_BUSY_CYCLES'] / 4:.2f},"
              f"{c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f},{c['SQ_INSTS_VALU'] / w:.0f},"
              f"{vmem / w:.0f},{miss / w:.2f},{miss / req if req else float('nan'):.4f}")


if __name__ == "__main__":
    a = sys.argv
    main(a[1], int(a[2]), int(a[3]), int(a[4]), int(a[5]), a[6:])
