"""Per-shape production rate against the live traffic ceilings (development tool).

For each shape, one resident batch and one plan: the production launch (rule order, and
optionally after rs_plan_tune), the kernel's no-lookup form, and the plan's read streams
alone + write streams alone (rs_plan_launch_ceiling), interleaved over rounds in one
process; every variant is warmed >= 30 ms before it is timed. Prints one JSON line per
shape with % of 8 TB/s (algorithmic bytes / mean launch time) for each.

shape spec: k,m,S,stripes[,erase[,layout[,order]]]   erase: '-' = encode, 'none' = all present,
            or '+'-joined indices (5, 0+3+7+12); layout: 'pitch' (StripeBatch, 256-B
            pitch, default), 'split' (upstream Split layout: object b's shard i at
            base + (b*n + i)*S from an odd base, every shard at its own byte offset when
            S is odd), 'contig' (the same from an aligned base) or 'readall' (Split of an
            io.ReadAll body: data shards at pitch S in page-aligned bodies, parity in
            64-B AllocAligned buffers; device.StripeBatch); 'planar:P' / 'pitch:P' set
            the shard pitch to P bytes; order: the plan's launches pinned to that tile order
            / kernel form (device.ORDER_NAMES, rs_plan_set_orders) instead of the rule's
usage: python tools/ceiling_sweep.py --shape 10,4,1048576,256,5 --shape ... [--tune 1]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import torch  # noqa: E402

from callfs_amd.device import Plan, StripeBatch  # noqa: E402

PEAK = 8000.0


def launch_ms(fn, stream, reps, warm_ms=30.0):
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < warm_ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / reps


def build(k, m, S, B, layout, dev):
    n = k + m
    if layout in ("split", "contig"):
        total = B * n * S
        buf = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device=dev)
        # split: odd base, so with odd S every shard sits at its own offset; contig: the
        # same pitch = S layout from an aligned base (aligned shards when 16 | S)
        base = buf.data_ptr() + (1 if layout == "split" else 0)
        ptrs = [base + (b * n + i) * S for b in range(B) for i in range(n)]
        return buf, ptrs
    # "planar:P" / "pitch:P": that layout at an explicit shard pitch of P bytes
    name, _, p = layout.partition(":")
    sb = StripeBatch(k, m, S, B, dev,
                     layout=name if name in ("readall", "planar", "shardmajor") else "pitch",
                     pitch=int(p) if p else None)
    sb.fill_random(0xCA11F5)
    return sb, sb.pointers()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tune", type=int, default=0)
    ap.add_argument("--fresh", type=int, default=0,
                    help="1: decodes rebuild the erased shards into fresh buffers instead of in place")
    ap.add_argument("--only", default="",
                    help="comma-separated variants to time (prod,tuned,nolookup,read,write); "
                         "default all (rocprofv3 --pmc passes time only prod)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for spec in a.shape:
        f = spec.split(",")
        k, m, S, B = (int(x) for x in f[:4])
        erase = f[4] if len(f) > 4 else "-"
        layout = f[5] if len(f) > 5 else "pitch"
        pin = f[6] if len(f) > 6 else ""
        n = k + m
        if erase not in ("-", "none") and (len({int(x) for x in erase.split("+")}) > m or
                                           max(int(x) for x in erase.split("+")) >= n):
            # (round 4's layout probe asked for 3 erasures of RS(4,2) and died in
            # rs_plan_create: an unrecoverable shape is reported, not run)
            print(json.dumps({"shape": spec, "skipped": f"erase {erase} is not recoverable "
                                                        f"for RS({k},{m})"}), flush=True)
            continue
        holder, ptrs = build(k, m, S, B, layout, dev)
        enc = Plan(k, m, S, B, ptrs)
        enc.launch(stream)
        if erase == "-":
            present = None
        elif erase == "none":
            present = [True] * n
        else:
            er = {int(x) for x in erase.split("+")}
            present = [i not in er for i in range(n)]
        fresh_buf = None
        if present is not None and a.fresh and not all(present):
            # the erased shards rebuilt into a region of their own (64-B pitch, 256-B aligned),
            # as upstream Reconstruct allocates missing shards (bench.py --decode-into fresh)
            from callfs_amd.device import _aligned_empty
            miss = [i for i in range(n) if not present[i]]
            fp = -(-S // 64) * 64
            fresh_buf = _aligned_empty((B, len(miss), fp), 256, dev)
            ptrs = list(ptrs)
            for b in range(B):
                for j, i in enumerate(miss):
                    ptrs[b * n + i] = fresh_buf[b, j].data_ptr()
        plan = enc if present is None else Plan(k, m, S, B, ptrs, present=present)
        if pin:
            from callfs_amd import _native as N
            try:
                plan.set_orders([pin] * int(N.lib.rs_plan_groups(plan.handle)))
            except N.NativeError as e:  # not offered for this launch: reported, not run
                print(json.dumps({"shape": spec, "skipped": f"order {pin}: {e}"}), flush=True)
                del plan, enc, holder, fresh_buf
                torch.cuda.empty_cache()
                continue
        variants = {"prod": lambda: plan.launch(stream)}
        orders = None
        if a.tune:
            tuned = Plan(k, m, S, B, ptrs, present=present)
            orders = tuned.tune(stream=stream)
            variants["tuned"] = lambda: tuned.launch(stream)
        for mode in ("nolookup", "read", "write"):
            variants[mode] = (lambda md: lambda: plan.launch_ceiling(md, stream))(mode)
        if a.only:
            keep = set(a.only.split(","))
            variants = {v: f for v, f in variants.items() if v in keep}
        t = {v: [] for v in variants}
        for r in range(a.rounds):
            names = list(variants)
            names = names[r % len(names):] + names[:r % len(names)]
            for v in names:
                t[v].append(launch_ms(variants[v], stream, a.reps))
        plan.corrupt(stream)
        plan.launch(stream)
        bad = plan.corrupt(stream)
        nb = plan.bytes
        best = {v: min(x) for v, x in t.items()}
        pct = {v: round(nb / (ms * 1e-3) / 1e9 / PEAK * 100, 2) for v, ms in best.items()
               if v not in ("read", "write")}
        if "read" in best and "write" in best:
            rw = nb / ((best["read"] + best["write"]) * 1e-3) / 1e9 / PEAK * 100
            pct["read+write"] = round(rw, 2)
            if "prod" in pct:
                pct["prod/read+write"] = round(pct["prod"] / rw, 4)
        out = {"shape": spec, "k": k, "m": m, "S": S, "stripes": B, "erase": erase,
               "layout": layout, "order": pin or "rule", "bytes": nb, "pct_of_8TBs": pct,
               "ms": {v: round(x, 4) for v, x in best.items()}, "tuned_orders": orders,
               "verify_after": bool(bad)}
        print(json.dumps(out), flush=True)
        del plan, enc, holder, fresh_buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
