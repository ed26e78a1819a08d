"""Summarize a tools/profile.sh output dir into profiles/<round>/ (kernel stats + HBM
traffic from the separate FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected)."""
import csv
import json
import os
import shutil
import statistics
import sys


def _per_op(rows, key):
    """bench.py launches the encode and the decode plan strictly alternately (both are
    rs_apply_lds<R=4> for RS(10,4) erase 4, so one kernel name): even dispatches of the
    hot kernel are encodes, odd ones decodes."""
    rows = sorted(rows, key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
    return [key(r) for r in rows[0::2]], [key(r) for r in rows[1::2]]


def main(src, dst, k=10, m=4, S=1 << 20, B=256, erase=(0, 1, 2, 3), kernel="rs_apply"):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
    ks = [r for r in rows if kernel in r["Name"]][0]
    algo = B * S * (k + m)
    out = {
        "config": {"k": k, "m": m, "shard_bytes": S, "stripes": B, "erase": list(erase)},
        "kernel": ks["Name"],
        "kernel_stats": {"calls": int(ks["Calls"]), "avg_ns": float(ks["AverageNs"]),
                         "min_ns": float(ks["MinNs"]), "max_ns": float(ks["MaxNs"])},
        "source": ("rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE and --pmc WRITE_SIZE in "
                   "separate passes of bench.py (tools/profile.sh); encode = even, decode = odd "
                   "dispatches of the hot kernel (bench.py alternates the two plans)"),
        "correction": ("gfx950: FETCH_SIZE counts half the bytes of 16-B/lane streaming reads "
                       "(MI355X_MICROARCH.md, HBM) -> fetch bytes = 2*FETCH_SIZE*1024; WRITE_SIZE "
                       "is exact for 16-B/lane stores"),
        "algorithmic_bytes_per_launch": algo,
    }
    trace = os.path.join(src, "kt", "kt_kernel_trace.csv")
    rows = list(csv.DictReader(open(trace)))
    hot = [r for r in rows if kernel in r.get("Kernel_Name", "")]
    with open(os.path.join(dst, "kernel_trace_rs_apply.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(hot[0].keys()))
        w.writeheader()
        w.writerows(hot)
    enc_d, dec_d = _per_op(hot, lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = {}
    for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        f = os.path.join(src, sub, f"{sub}_counter_collection.csv")
        v = [r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
        pmc[name] = _per_op(v, lambda r: float(r["Counter_Value"]))
    for op, durs, idx in (("encode", enc_d, 0), ("decode", dec_d, 1)):
        ds = sorted(durs)
        fetch = statistics.median(pmc["FETCH_SIZE"][idx])
        write = statistics.median(pmc["WRITE_SIZE"][idx])
        fetch_b, write_b = fetch * 1024 * 2, write * 1024
        # grids of > 2 x ~4 GiB of traffic run as several dispatches per plan launch
        # (rs_kernels.hip slice_tiles): scale per-dispatch counters to one launch
        slices = max(1, round(algo / (fetch_b + write_b)))
        avg = sum(ds) / len(ds) * slices
        out[op] = {
            "dispatches": len(ds),
            "avg_ns": avg,
            "median_ns": ds[len(ds) // 2] * slices,
            "achieved_gbs": algo / avg,
            "frac_of_8tbs": algo / avg / 8000.0,
            "FETCH_SIZE_kib": fetch, "WRITE_SIZE_kib": write,
            "pmc_dispatches": [len(pmc["FETCH_SIZE"][idx]), len(pmc["WRITE_SIZE"][idx])],
            "fetch_bytes_per_launch": fetch_b * slices,
            "write_bytes_per_launch": write_b * slices,
            "dispatches_per_launch": slices,
        }
        out[f"{op}_bytes_per_launch"] = (fetch_b + write_b) * slices
    json.dump(out, open(os.path.join(dst, "hbm_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    # usage: summarize_profile.py <profile dir> <dst dir> [k m shard_bytes stripes erase]
    a = sys.argv[1:]
    extra = [int(x) for x in a[2:6]]
    if len(a) > 6:
        extra.append(tuple(int(x) for x in a[6].split(",")))
    main(a[0], a[1], *extra)
