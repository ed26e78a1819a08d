"""Read- and write-stream alignment probe (development tool, DESIGN.md §5 Split layout).

For each shape: the plan's write streams alone (rs_plan_launch_ceiling RS_CEIL_WRITE,
16-B-aligned rows as the production stores) against the same streams written from each
row's first 64 / 128 / 256-B boundary (RS_CEIL_WRITE_AL*), interleaved over rounds in
one process. Prints % of 8 TB/s of the written bytes per variant.
usage: python tools/write_align_probe.py --shape k,m,S,stripes[,layout] ...
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tools"))

import torch  # noqa: E402

from callfs_amd.device import Plan  # noqa: E402
from ceiling_sweep import build, launch_ms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for spec in a.shape:
        f = spec.split(",")
        k, m, S, B = (int(x) for x in f[:4])
        layout = f[4] if len(f) > 4 else "pitch"
        holder, ptrs = build(k, m, S, B, layout, dev)
        plan = Plan(k, m, S, B, ptrs)
        modes = ["write", "write64", "write128", "write256", "read", "read64", "read128",
                 "read256"]
        t = {md: [] for md in modes}
        for r in range(a.rounds):
            for md in modes[r % 8:] + modes[:r % 8]:
                t[md].append(launch_ms(lambda: plan.launch_ceiling(md, stream), stream, a.reps))
        wb, rb = m * S * B, k * S * B
        pct = {md: round((rb if md.startswith("read") else wb) / (min(x) * 1e-3) / 1e9 / 80.0, 2)
               for md, x in t.items()}
        print(json.dumps({"shape": spec, "written_bytes": wb, "pct_of_8TBs": pct}), flush=True)
        del plan, holder
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
