"""Bit-sliced kernel against the rule's kernel (development tool).

For each shape: one resident batch, the rule's plan and one plan per pinned bit-sliced order
("bs", "bs-q8", "bs-x32", "bs-g2"); the pinned plans' outputs must equal the rule's bytes
(the rule's kernels are pinned to the oracle by tests/test_gpu_parity.py), then each plan is
timed in rotated rounds. One JSON line per shape: % of 8 TB/s (algorithmic bytes / mean
launch time) per variant.

shape spec: k,m,S,stripes[,erase]   erase: '-' encode, 'none' (read-only Verify), or '+'-joined
erased indices
usage: python tools/bs_probe.py --shape 32,16,1048576,64 [--orders bs,bs-q8]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import torch  # noqa: E402

from callfs_amd import _native as N  # noqa: E402
from callfs_amd.device import Plan, StripeBatch  # noqa: E402

PEAK = 8000.0


def launch_ms(fn, stream, reps, warm_ms=30.0):
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < warm_ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", required=True)
    ap.add_argument("--orders", default="bs,bs-q8,bs-x32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--layout", default="planar")
    ap.add_argument("--fresh", type=int, default=0,
                    help="1: decodes rebuild the erased shards into fresh buffers")
    ap.add_argument("--tune", type=int, default=0, help="1: also an rs_plan_tune plan")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for spec in a.shape:
        f = spec.split(",")
        k, m, S, B = (int(x) for x in f[:4])
        erase = f[4] if len(f) > 4 else "-"
        n = k + m
        sb = StripeBatch(k, m, S, B, dev, layout=a.layout)
        sb.fill_random(0xB17)
        ptrs = sb.pointers()
        Plan(k, m, S, B, ptrs).launch(stream)  # the rule's parity: every stripe consistent
        torch.cuda.synchronize()
        ref = sb.gather()
        present = None
        lost = list(range(k, n))
        if erase != "-":  # 'none': every shard present (a download's Verify, read-only)
            lost = [] if erase == "none" else sorted({int(x) for x in erase.split("+")})
            present = [i not in lost for i in range(n)]
        fresh = None
        if a.fresh and present is not None:
            # the erased shards rebuilt into buffers of their own (64-B pitch, 256-B aligned),
            # as upstream Reconstruct allocates missing shards (bench.py --decode-into fresh)
            from callfs_amd.device import _aligned_empty
            fp = -(-S // 64) * 64
            fresh = _aligned_empty((B, len(lost), fp), 256, dev)
            ptrs = list(ptrs)
            for b in range(B):
                for j, i in enumerate(lost):
                    ptrs[b * n + i] = fresh[b, j].data_ptr()
        rule = Plan(k, m, S, B, ptrs, present=present)
        plans = {"rule": rule}
        out = {"shape": spec, "k": k, "m": m, "S": S, "stripes": B, "erase": erase,
               "layout": a.layout, "fresh": fresh is not None}

        def exact(p):
            if fresh is not None:
                fresh.zero_()
            else:
                for i in lost:
                    sb.zero_shard(i)
            p.launch(stream)
            torch.cuda.synchronize()
            if fresh is not None:
                ok = all(torch.equal(fresh[:, j, :S], ref[:, i]) for j, i in enumerate(lost))
            else:
                ok = bool(torch.equal(sb.gather(), ref))
            return ok and not p.corrupt(stream)

        out["bit_exact"] = {"rule": exact(rule)}
        for o in a.orders.split(","):
            p = Plan(k, m, S, B, ptrs, present=present)
            try:
                p.set_orders([o] * int(N.lib.rs_plan_groups(p.handle)))
            except N.NativeError as e:
                out.setdefault("skipped", {})[o] = str(e)
                continue
            t0 = time.perf_counter()
            p.launch(stream)  # a pinned bit-sliced order waits for its compile
            torch.cuda.synchronize()
            out.setdefault("first_launch_s", {})[o] = round(time.perf_counter() - t0, 2)
            out["bit_exact"][o] = exact(p)
            plans[o] = p
        if a.tune:
            tp = Plan(k, m, S, B, ptrs, present=present)
            out["tuned_orders"] = tp.tune(stream=stream)
            out["bit_exact"]["tuned"] = exact(tp)
            plans["tuned"] = tp
        t = {v: [] for v in plans}
        for r in range(a.rounds):
            names = list(plans)
            names = names[r % len(names):] + names[:r % len(names)]
            for v in names:
                t[v].append(launch_ms(lambda: plans[v].launch(stream), stream, a.reps))
        nb = rule.bytes
        out["pct_of_8TBs"] = {v: round(nb / (min(x) * 1e-3) / 1e9 / PEAK * 100, 2) for v, x in t.items()}
        print(json.dumps(out), flush=True)
        del plans, rule, sb, ref, fresh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
