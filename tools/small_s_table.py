"""Table of tools/small_s_probe.sh: % of 8 TB/s per variant and the L2's mean memory read
latency (TCC_EA0_RDREQ_LEVEL_sum / TCC_EA0_RDREQ_sum, cycles; Little's law) of that
variant's kernel. usage: python tools/small_s_table.py <dir>"""
import csv
import glob
import os
import re
import sys


def pmc(d):
    tot = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "rs_apply" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


def main(base):
    print("shape,variant,pct_8TBs,read_latency_cycles")
    for log in sorted(glob.glob(os.path.join(base, "time_*.log"))):
        k, m, S = os.path.basename(log)[5:-4].split("_")
        for line in open(log):
            mm = re.match(r"(prod dispatch|persist \d)\s+[\d.]+\s+[\d.]+\s+[\d.]+\s+([\d.]+)", line)
            if not mm:
                continue
            v = mm.group(1)
            c = pmc(os.path.join(base, f"pmc_{k}_{m}_{S}_{v.replace(' ', '_')}"))
            lat = c["TCC_EA0_RDREQ_LEVEL_sum"] / c["TCC_EA0_RDREQ_sum"] if c.get("TCC_EA0_RDREQ_sum") else float("nan")
            print(f"RS({k},{m}) S={S},{v},{mm.group(2)},{lat:.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
