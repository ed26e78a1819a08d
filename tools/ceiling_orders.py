"""Read-alone and write-alone stream rates of a plan's traffic in each tile order
(rs_plan_launch_ceiling modes 1 / 2 after Plan.set_orders; development tool). Separates
what an order does to HBM reads from what it does to writes.
shape spec as tools/ceiling_sweep.py: k,m,S,stripes[,erase[,layout]]
usage: python tools/ceiling_orders.py --orders consecutive,g2,q8 --shape 10,4,6710887,256,-,planar
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
    ap.add_argument("--rounds", type=int, default=2)
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
        present = None
        if erase == "none":
            present = [True] * n
        elif erase != "-":
            er = {int(x) for x in erase.split("+")}
            present = [i not in er for i in range(n)]
        p = Plan(k, m, S, B, ptrs, present=present)
        nr = k if present is None else k  # inputs read
        nw = (m if present is None else n - sum(present))
        res = {}
        for rnd in range(a.rounds):
            for o in a.orders.split(","):
                try:
                    p.set_orders([o])
                except N.NativeError:
                    continue
                for mode in ("read", "write"):
                    ms = launch_ms(lambda: p.launch_ceiling(mode, stream), stream, a.reps)
                    res.setdefault(o, {}).setdefault(mode, []).append(ms)
        out = {}
        for o, d in res.items():
            rd = B * nr * S / min(d["read"]) / 1e6
            wr = B * nw * S / min(d["write"]) / 1e6
            tot = B * (nr + nw) * S / (min(d["read"]) + min(d["write"])) / 1e6
            out[o] = {"read_GBs": round(rd), "write_GBs": round(wr), "r+w_pct": round(tot / 80, 2)}
        print(json.dumps({"shape": spec, "orders": out}), flush=True)
        del p, holder
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
