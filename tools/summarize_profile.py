"""Summarize a tools/profile.sh output dir into profiles/<round>/ (kernel stats + HBM
traffic from the separate FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected)."""
import csv
import json
import os
import shutil
import statistics
import sys


def main(src, dst, k=10, m=4, S=1 << 20, B=256, kernel="rs_apply_lds"):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
    ks = [r for r in rows if kernel in r["Name"]][0]
    vals = {}
    for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        f = os.path.join(src, sub, f"{sub}_counter_collection.csv")
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
        vals[name] = (statistics.median(v), len(v))
    fetch_b = vals["FETCH_SIZE"][0] * 1024 * 2
    write_b = vals["WRITE_SIZE"][0] * 1024
    # grids of > 2 x ~2 GiB of traffic run as several dispatches per plan launch
    # (rs_kernels.hip slice_tiles): scale per-dispatch counters to one launch
    algo = B * S * (k + m)
    slices = max(1, round(algo / (fetch_b + write_b)))
    fetch_b *= slices
    write_b *= slices
    out = {
        "config": {"k": k, "m": m, "shard_bytes": S, "stripes": B},
        "kernel": ks["Name"],
        "kernel_trace": {"calls": int(ks["Calls"]), "avg_ns": float(ks["AverageNs"]),
                         "min_ns": float(ks["MinNs"]), "max_ns": float(ks["MaxNs"])},
        "source": ("rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE and --pmc WRITE_SIZE in "
                   "separate passes of bench.py (tools/profile.sh); medians over %d / %d dispatches"
                   % (vals["FETCH_SIZE"][1], vals["WRITE_SIZE"][1])),
        "FETCH_SIZE_kib": vals["FETCH_SIZE"][0],
        "WRITE_SIZE_kib": vals["WRITE_SIZE"][0],
        "correction": ("gfx950: FETCH_SIZE counts half the bytes of 16-B/lane streaming reads "
                       "(MI355X_MICROARCH.md, HBM) -> fetch bytes = 2*FETCH_SIZE*1024; WRITE_SIZE "
                       "is exact for 16-B/lane stores"),
        "fetch_bytes_per_launch": fetch_b,
        "write_bytes_per_launch": write_b,
        "encode_bytes_per_launch": fetch_b + write_b,
        "algorithmic_bytes_per_launch": algo,
        "dispatches_per_launch": slices,
    }
    trace = os.path.join(src, "kt", "kt_kernel_trace.csv")
    if os.path.exists(trace):  # per-dispatch rows of the hot kernel
        rows = list(csv.DictReader(open(trace)))
        hot = [r for r in rows if kernel in r.get("Kernel_Name", "")]
        if hot:
            with open(os.path.join(dst, "kernel_trace_rs_apply.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(hot[0].keys()))
                w.writeheader()
                w.writerows(hot)
            durs = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in hot)
            out["kernel_trace"]["median_ns"] = durs[len(durs) // 2]
    json.dump(out, open(os.path.join(dst, "hbm_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    # usage: summarize_profile.py <profile dir> <dst dir> [k m shard_bytes stripes]
    a = sys.argv[1:]
    extra = [int(x) for x in a[2:6]]
    main(a[0], a[1], *extra)
