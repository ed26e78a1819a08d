"""Summarise tools/pmc_sweep.sh output: per shape, the production kernel's counters per
dispatch (rs_apply_lds / rs_apply_vec instances, NOMATH and stream kernels excluded), with
the gfx950 FETCH_SIZE correction (x2, MI355X_MICROARCH.md) and bytes against the
algorithmic bytes per launch. usage: python tools/pmc_sweep_table.py gpurun_out/<tag>"""
import csv
import glob
import json
import os
import statistics
import sys


def prod_kernel(name):
    # the sweep's --only prod launches production kernels only (no ceiling forms)
    return "rs_apply_lds" in name or "rs_apply_vec" in name


def main(d):
    rows = []
    for shp in sorted(glob.glob(os.path.join(d, "s*.shape")), key=lambda p: int(os.path.basename(p)[1:-6])):
        i = os.path.basename(shp)[1:-6]
        spec = open(shp).read().strip()
        vals = {}
        nbytes = None
        for p in range(6):
            log = os.path.join(d, f"s{i}_p{p}.log")
            if nbytes is None and os.path.exists(log):
                for ln in open(log):
                    if ln.startswith("{"):
                        nbytes = json.loads(ln)["bytes"]
            for f in glob.glob(os.path.join(d, f"s{i}_p{p}", "**", "*counter_collection.csv"), recursive=True):
                per = {}
                for r in csv.DictReader(open(f)):
                    if not prod_kernel(r["Kernel_Name"]):
                        continue
                    key = (r["Dispatch_Id"], r["Counter_Name"])
                    per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
                by = {}
                for (disp, c), v in per.items():
                    by.setdefault(c, []).append(v)
                for c, v in by.items():
                    vals[c] = statistics.median(v)
        out = {"shape": spec, "algorithmic_bytes": nbytes}
        if "FETCH_SIZE" in vals:
            out["fetch_bytes"] = 2 * vals["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in vals:
            out["write_bytes"] = vals["WRITE_SIZE"] * 1024
        if nbytes and "fetch_bytes" in out and "write_bytes" in out:
            out["traffic_over_algorithmic"] = round((out["fetch_bytes"] + out["write_bytes"]) / nbytes, 4)
        if vals.get("TCC_EA0_RDREQ_LEVEL_sum") and vals.get("TCC_EA0_RDREQ_sum"):
            # Little's law: mean read requests outstanding x cycles / requests = mean
            # memory-side read latency in L2 cycles
            out["read_latency_tcc_cycles"] = round(vals["TCC_EA0_RDREQ_LEVEL_sum"] / vals["TCC_EA0_RDREQ_sum"], 1)
        if vals.get("TCC_EA0_WRREQ_LEVEL_sum") and vals.get("TCC_EA0_WRREQ_sum"):
            out["write_latency_tcc_cycles"] = round(vals["TCC_EA0_WRREQ_LEVEL_sum"] / vals["TCC_EA0_WRREQ_sum"], 1)
        out["counters"] = vals
        rows.append(out)
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
