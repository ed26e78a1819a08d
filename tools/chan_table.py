"""Table of tools/jobs.sh chan_probe's memory-side counters (development tool).

Per shape (in --shape order) and variant (the plan's launch, its read streams alone, its
write streams alone): µs per launch under the profiler, average read / write latency in
cycles (REQ_LEVEL / REQ: requests in flight summed per cycle over requests), the fraction of
channel-cycles stalled on DRAM credits (counter / (16 channels x 8 XCDs x GUI cycles per
XCD)), and the fraction of requests that reach DRAM. Dispatches are grouped into runs of
one kernel and grid; each run's median is taken, and runs of >= 3 dispatches are dealt out
three per shape (prod, read, write), as tools/ceiling_sweep.py issues them.
usage: python tools/chan_table.py gpurun_out/chan_<tag> > table.csv
"""
import csv
import glob
import json
import os
import statistics
import sys

CHANNELS = 16 * 8


def runs(path):
    out, key, cur = [], None, []
    rows = {}
    for r in csv.DictReader(open(path)):
        if "rs_apply" not in r["Kernel_Name"] and "rs_stream" not in r["Kernel_Name"]:
            continue
        d = rows.setdefault(int(r["Dispatch_Id"]), {
            "kern": r["Kernel_Name"].split("<")[0].split("::")[-1], "grid": r["Grid_Size"],
            "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    for _, d in sorted(rows.items()):
        k = (d["kern"], d["grid"])
        if k != key and cur:
            out.append(cur)
            cur = []
        key = k
        cur.append(d)
    if cur:
        out.append(cur)
    med = []
    for c in out:
        if len(c) < 3:
            continue
        m = {"kern": c[0]["kern"], "n": len(c)}
        for f in c[0]:
            if f not in ("kern", "grid"):
                m[f] = statistics.median(x[f] for x in c)
        med.append(m)
    return med


def main():
    d = sys.argv[1]
    shapes = [json.loads(x) for x in open(os.path.join(d, "p1.log")) if x.startswith('{"shape"')]
    passes = [runs(p) for p in sorted(glob.glob(os.path.join(d, "p*", "p*_counter_collection.csv")))]
    w = csv.writer(sys.stdout)
    w.writerow(["shape", "variant", "kernel", "us", "GBps_alg", "rd_lat_cyc", "wr_lat_cyc",
                "wr_dram_credit_stall", "rd_dram_credit_stall", "wr_stall", "tag_stall",
                "wr_to_dram", "rd_to_dram", "bytes_per_wrreq", "bytes_per_rdreq"])
    for si, sh in enumerate(shapes):
        k, m, S, B = sh["k"], sh["m"], sh["S"], sh["stripes"]
        nb = sh["bytes"]
        for vi, var in enumerate(("prod", "read", "write")):
            got = {}
            for p in passes:
                if 3 * si + vi < len(p):
                    got.update(p[3 * si + vi])
            if not got:
                continue
            cyc = got.get("GRBM_GUI_ACTIVE", 0) / 8 or float("nan")

            def g(c):
                return got.get(c, float("nan"))
            rows_w = m if sh["erase"] == "-" else len(sh["erase"].split("+"))
            wbytes = B * rows_w * S
            rbytes = nb - wbytes
            alg = {"prod": nb, "read": rbytes, "write": wbytes}[var]
            w.writerow([sh["shape"], var, got["kern"], round(got["ns"] / 1e3, 1),
                        round(alg / got["ns"], 1),
                        round(g("TCC_EA0_RDREQ_LEVEL") / g("TCC_EA0_RDREQ"), 1) if g("TCC_EA0_RDREQ") else "",
                        round(g("TCC_EA0_WRREQ_LEVEL") / g("TCC_EA0_WRREQ"), 1) if g("TCC_EA0_WRREQ") else "",
                        round(g("TCC_EA0_WRREQ_DRAM_CREDIT_STALL") / (CHANNELS * cyc), 4),
                        round(g("TCC_EA0_RDREQ_DRAM_CREDIT_STALL") / (CHANNELS * cyc), 4),
                        round(g("TCC_EA0_WRREQ_STALL") / (CHANNELS * cyc), 4),
                        round(g("TCC_TAG_STALL") / (CHANNELS * cyc), 4),
                        round(g("TCC_EA0_WRREQ_DRAM") / g("TCC_EA0_WRREQ"), 4) if g("TCC_EA0_WRREQ") else "",
                        round(g("TCC_EA0_RDREQ_DRAM") / g("TCC_EA0_RDREQ"), 4) if g("TCC_EA0_RDREQ") else "",
                        round(wbytes / g("TCC_EA0_WRREQ"), 1) if var != "read" and g("TCC_EA0_WRREQ") else "",
                        round(rbytes / g("TCC_EA0_RDREQ"), 1) if var != "write" and g("TCC_EA0_RDREQ") else ""])


if __name__ == "__main__":
    main()
