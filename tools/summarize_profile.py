"""Summarize a tools/jobs.sh profile output dir into profiles/<round>/ (kernel stats + HBM
traffic from the separate FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected)."""
import csv
import json
import os
import shutil
import statistics
import sys


def _order(rows):
    return sorted(rows, key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))


def _bench_steps(log):
    """`steps` of the bench JSON line in a profiled bench.py log."""
    for ln in reversed(open(log).read().splitlines()):
        if ln.startswith("{") and '"steps"' in ln:
            return int(json.loads(ln)["steps"])
    raise SystemExit(f"no bench line in {log}")


def _per_op(rows, key, steps, slices):
    """The timed region is the tail of the trace: bench.py launches the encode and the
    decode plan strictly alternately, `steps` times each, each plan launch being `slices`
    dispatches. Dispatches before it (round-trip check, rs_plan_tune's candidate orders,
    warmup) are dropped. Returns the per-dispatch values of the encode and decode
    launches."""
    tail = _order(rows)[-2 * steps * slices:]
    enc, dec = [], []
    for i in range(0, len(tail), slices):
        (enc if (i // slices) % 2 == 0 else dec).extend(key(r) for r in tail[i:i + slices])
    return enc, dec


def main(src, dst, k=10, m=4, S=1 << 20, B=256, erase=(0, 1, 2, 3), layout="planar",
         kernel="rs_apply"):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    algo = B * S * (k + m)
    trace = os.path.join(src, "kt", "kt_kernel_trace.csv")
    allrows = _order(r for r in csv.DictReader(open(trace)) if kernel in r.get("Kernel_Name", ""))
    hot_name = allrows[-2]["Kernel_Name"]  # the encode plan's instance in the timed steps
    rows = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
    ks = [r for r in rows if r["Name"] == hot_name][0]
    out = {
        "config": {"k": k, "m": m, "shard_bytes": S, "stripes": B,
                   **({"layout": layout} if layout != "pitch" else {}), "erase": list(erase)},
        "kernel": ks["Name"],
        "kernel_stats": {"calls": int(ks["Calls"]), "avg_ns": float(ks["AverageNs"]),
                         "min_ns": float(ks["MinNs"]), "max_ns": float(ks["MaxNs"])},
        "source": ("rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE and --pmc WRITE_SIZE in "
                   "separate passes of bench.py (tools/jobs.sh profile); the timed steps are the "
                   "last 2 x steps plan launches of the trace, alternately encode and decode "
                   "(earlier dispatches: round-trip check, rs_plan_tune candidates, warmup); "
                   "kernel_stats covers every dispatch of the instance, tuning included"),
        "correction": ("gfx950: FETCH_SIZE counts half the bytes of 16-B/lane streaming reads "
                       "(MI355X_MICROARCH.md, HBM) -> fetch bytes = 2*FETCH_SIZE*1024; WRITE_SIZE "
                       "is exact for 16-B/lane stores"),
        "algorithmic_bytes_per_launch": algo,
    }
    with open(os.path.join(dst, "kernel_trace_rs_apply.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(allrows[0].keys()))
        w.writeheader()
        w.writerows(allrows)
    pmc_rows = {}
    for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        f = os.path.join(src, sub, f"{sub}_counter_collection.csv")
        pmc_rows[name] = _order(r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"])
    # grids of > 2 x ~4 GiB of traffic run as several dispatches per plan launch
    # (rs_kernels.hip slice_tiles): dispatches per launch from the last dispatch's bytes
    last_b = (2 * 1024 * float(pmc_rows["FETCH_SIZE"][-1]["Counter_Value"])
              + 1024 * float(pmc_rows["WRITE_SIZE"][-1]["Counter_Value"]))
    slices = max(1, round(algo / last_b))
    steps = _bench_steps(os.path.join(src, "bench_kt.log"))
    pmc_steps = _bench_steps(os.path.join(src, "bench_fetch.log"))
    enc_d, dec_d = _per_op(allrows, lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                           steps, slices)
    pmc = {name: _per_op(v, lambda r: float(r["Counter_Value"]), pmc_steps, slices)
           for name, v in pmc_rows.items()}
    tail = allrows[-2 * steps * slices:]
    hot_name = tail[0]["Kernel_Name"]
    ks = [r for r in rows if r["Name"] == hot_name][0]
    out["kernel"] = hot_name
    out["kernel_stats"] = {"calls": int(ks["Calls"]), "avg_ns": float(ks["AverageNs"]),
                           "min_ns": float(ks["MinNs"]), "max_ns": float(ks["MaxNs"])}
    out["timed_dispatches"] = {"encode_kernel": hot_name, "decode_kernel": tail[slices]["Kernel_Name"],
                               "steps": steps, "pmc_steps": pmc_steps}
    for op, durs, idx in (("encode", enc_d, 0), ("decode", dec_d, 1)):
        ds = sorted(durs)
        fetch = statistics.median(pmc["FETCH_SIZE"][idx])
        write = statistics.median(pmc["WRITE_SIZE"][idx])
        fetch_b, write_b = fetch * 1024 * 2, write * 1024
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
    # usage: summarize_profile.py <profile dir> <dst dir> [k m shard_bytes stripes erase layout kernel]
    a = sys.argv[1:]
    extra = [int(x) for x in a[2:6]]
    if len(a) > 6:
        extra.append(tuple(int(x) for x in a[6].split(",")))
    if len(a) > 7:
        extra.append(a[7])
    if len(a) > 8:  # the kernel name filter: "rs_bs" for the bit-sliced kernels
        extra.append(a[8])
    main(a[0], a[1], *extra)
