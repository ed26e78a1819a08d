"""Device-resident decode efficiency per erasure pattern (development tool, not product).

Times rs_plan launches (HIP events on the launch stream) for an encode plan and for
decode plans of several erasure patterns over one resident StripeBatch, and prints the
algorithmic bytes per launch (rs_plan_bytes: k valid reads + compared parity reads +
missing-shard writes per stripe) over the median launch time.

The all-present pattern is upstream's Verify on every download (codec.go:59): m verify
rows, no writes. One erasure of a data shard = 1 write row + m-1 verify rows.

usage: python tools/decode_sweep.py [--k 10 --m 4 --shard-bytes 1048576 --stripes 256]
"""
import argparse
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import torch  # noqa: E402

from callfs_amd.device import Plan, StripeBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--shard-bytes", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--patterns", default="enc;;5;0,3,7,12;0,1,2,3;10,11,12,13;0;13")
    ap.add_argument("--tune", type=int, default=0,
                    help="1: also time a second plan per pattern tuned by rs_plan_tune")
    a = ap.parse_args()
    k, m, S, B = a.k, a.m, a.shard_bytes, a.stripes
    dev = torch.device("cuda", 0)
    sb = StripeBatch(k, m, S, B, dev)
    sb.fill_random(0xCA11F5)
    stream = torch.cuda.current_stream(dev)
    enc = Plan.for_batch(sb)
    enc.launch(stream)  # consistent parity: verify rows must pass
    plans = []
    orders = {}
    for p in a.patterns.split(";"):
        if p == "enc":
            plans.append(("encode", enc))
            present = None
            name = "encode"
        else:
            erase = sorted({int(x) for x in p.split(",") if x})
            present = [i not in erase for i in range(k + m)]
            name = f"decode erase {erase}"
            plans.append((name, Plan.for_batch(sb, present=present)))
        if a.tune:
            tuned = Plan.for_batch(sb, present=present)
            orders[name + " (tuned)"] = tuned.tune(stream=stream)
            plans.append((name + " (tuned)", tuned))
    times = {name: [] for name, _ in plans}
    for rd in range(a.rounds):
        for j in range(len(plans)):
            name, pl = plans[(j + rd) % len(plans)]
            pl.launch(stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.iters):
                pl.launch(stream)
            e1.record(stream)
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.iters)
    for name, pl in plans:
        if pl is not enc and pl.corrupt(stream):
            raise SystemExit(f"{name}: verify flagged corruption on consistent data")
        med = statistics.median(times[name])
        gbs = pl.bytes / (med * 1e-3) / 1e9
        print(json.dumps({"k": k, "m": m, "S": S, "stripes": B, "plan": name,
                          "bytes_per_launch": pl.bytes, "median_ms": round(med, 4),
                          "GB/s": round(gbs, 1), "frac_8TBs": round(gbs / 8000, 4),
                          "object_GiB/s": round(B * k * S / (med * 1e-3) / 2**30, 1),
                          "tile_order": orders.get(name)}))


if __name__ == "__main__":
    main()
