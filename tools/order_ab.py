"""Tile-order / kernel-form A/B through rs_plan_set_orders (development tool).

For each shape, one resident batch and one plan per named order (Plan.set_orders: the
order of launch group 0; orders the kernel does not offer are skipped), timed
interleaved over rounds in one process, every variant warmed >= 30 ms first. Prints one
JSON line per shape with % of 8 TB/s (algorithmic bytes / best-round mean launch time).
shape spec as tools/ceiling_sweep.py: k,m,S,stripes[,erase[,layout]]
usage: python tools/order_ab.py --orders realign,stage,stage-x32 --shape 10,4,6710887,64,-,split
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tools"))

import torch  # noqa: E402

from callfs_amd import _native as N  # noqa: E402
from callfs_amd.device import Plan  # noqa: E402
from ceiling_sweep import build, launch_ms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", required=True)
    ap.add_argument("--orders", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for spec in a.shape:
        f = spec.split(",")
        k, m, S, B = (int(x) for x in f[:4])
        erase = f[4] if len(f) > 4 else "-"
        layout = f[5] if len(f) > 5 else "pitch"
        n = k + m
        holder, ptrs = build(k, m, S, B, layout, dev)
        Plan(k, m, S, B, ptrs).launch(stream)  # consistent parity for decodes
        present = None
        if erase == "none":
            present = [True] * n
        elif erase != "-":
            er = {int(x) for x in erase.split("+")}
            present = [i not in er for i in range(n)]
        plans = {}
        for name in ["rule"] + a.orders.split(","):
            p = Plan(k, m, S, B, ptrs, present=present)
            if name != "rule":
                try:
                    p.set_orders([name])
                except N.NativeError:
                    continue
            plans[name] = p
        t = {v: [] for v in plans}
        names = list(plans)
        for r in range(a.rounds):
            for v in names[r % len(names):] + names[:r % len(names)]:
                t[v].append(launch_ms(lambda: plans[v].launch(stream), stream, a.reps))
        nb = plans["rule"].bytes
        bad = {v: p.corrupt(stream) for v, p in plans.items()}
        pct = {v: round(nb / (min(x) * 1e-3) / 1e9 / 80.0, 2) for v, x in t.items()}
        print(json.dumps({"shape": spec, "bytes": nb, "pct_of_8TBs": pct,
                          "verify_flagged": [v for v, b in bad.items() if b]}), flush=True)
        del plans, holder
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
