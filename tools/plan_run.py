"""Launch one plan N times in a given order (development tool: the program rocprofv3 profiles
for PMC passes, tools/jobs.sh pmc_forms). shape spec as tools/ceiling_sweep.py.
usage: python tools/plan_run.py --shape 10,8,6710887,32,-,planar --order tri-q8 --launches 20"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tools"))

import torch  # noqa: E402

from callfs_amd.device import Plan  # noqa: E402
from ceiling_sweep import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", required=True)
    ap.add_argument("--order", default="none")
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    f = a.shape.split(",")
    k, m, S, B = (int(x) for x in f[:4])
    erase = f[4] if len(f) > 4 else "-"
    layout = f[5] if len(f) > 5 else "pitch"
    dev = torch.device("cuda", 0)
    holder, ptrs = build(k, m, S, B, layout, dev)
    present = None
    if erase != "-":
        er = set() if erase == "none" else {int(x) for x in erase.split("+")}
        present = [i not in er for i in range(k + m)]
        Plan(k, m, S, B, ptrs).launch()
    p = Plan(k, m, S, B, ptrs, present=present)
    if a.order != "none":
        p.set_orders([a.order] * int(__import__("callfs_amd")._native.lib.rs_plan_groups(p.handle)))
    for _ in range(a.launches):
        p.launch()
    torch.cuda.synchronize()
    print("plan_run ok", a.shape, a.order, "corrupt" if p.corrupt() else "clean")


if __name__ == "__main__":
    main()
