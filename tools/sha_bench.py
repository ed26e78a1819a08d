#!/usr/bin/env python3
"""Batched SHA-256 (ShardChecksum) throughput: GPU (device-resident shards, one lane
per message, msgs-per-wave variants) vs CPU hashlib (OpenSSL) threads on the same data."""
import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=4)
    p.add_argument("--shard-bytes", type=int, default=1 << 20)
    p.add_argument("--stripes", type=int, default=256)
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--cpu-threads", type=int, default=16)
    args = p.parse_args()
    import torch
    from callfs_amd.device import HashPlan, StripeBatch
    sb = StripeBatch(args.k, args.m, args.shard_bytes, args.stripes, torch.device("cuda:0"))
    sb.fill_random(7)
    ptrs, lens = sb.pointers(), [sb.S] * (sb.batch * sb.n)
    total = sum(lens)
    out = torch.empty(32 * len(ptrs), dtype=torch.uint8, device="cuda:0")
    res = {"messages": len(ptrs), "message_bytes": sb.S, "total_bytes": total}
    ref = None
    for mpw in [1, 2, 4, 8, 16, 64]:
        os.environ["CALLFS_SHA_MSGS_PER_WAVE"] = str(mpw)
        hp = HashPlan(ptrs, lens)
        hp.launch(out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().tobytes()
        ref = ref or got
        assert got == ref
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            hp.launch(out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        res[f"gpu_mpw{mpw}_GBps"] = round(total / (ms * 1e-3) / 1e9, 2)
        res[f"gpu_mpw{mpw}_ms"] = round(ms, 2)
        hp.close()
    # CPU: hashlib over host copies of a sample (releases the GIL for large buffers)
    ns = min(64, sb.batch)
    host = sb.buf[:ns, :, :sb.S].cpu().numpy()
    msgs = [host[b, i] for b in range(ns) for i in range(sb.n)]
    digs = [hashlib.sha256(x).digest() for x in msgs[:sb.n]]
    assert b"".join(digs) == ref[:32 * sb.n], "GPU digests != hashlib"
    with ThreadPoolExecutor(args.cpu_threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda x: hashlib.sha256(x).digest(), msgs))
        el = time.perf_counter() - t0
    res["cpu_threads"] = args.cpu_threads
    res["cpu_GBps"] = round(sum(x.nbytes for x in msgs) / el / 1e9, 2)
    t0 = time.perf_counter()
    for x in msgs[:56]:
        hashlib.sha256(x).digest()
    res["cpu_1thread_GBps"] = round(sum(x.nbytes for x in msgs[:56]) / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
