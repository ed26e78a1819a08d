#!/usr/bin/env python3
"""End-to-end (host memory in, host memory out) RS throughput through the C ABI.

configs[4]-style sweep: RS(k, m) objects of 4 KiB .. 64 MiB through Codec.encode
(Split + parity, codec.go:21-41) and Codec.decode with `--erase` shards missing
(Reconstruct + Verify + join, codec.go:45-78), i.e. including the pinned staging
copies and H2D/D2H over PCIe. `--threads` request threads share one Codec like the
Go server's request goroutines share one *Codec (erasure/manager.go:60).

Prints one JSON line per size: encode and decode GiB/s of object bytes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=16)
    p.add_argument("--m", type=int, default=4)
    p.add_argument("--sizes", default="4K,16K,64K,256K,1M,4M,16M,64M")
    p.add_argument("--erase", default="0,5,16,19")
    p.add_argument("--threads", type=int, default=1)
    p.add_argument("--seconds", type=float, default=1.0, help="time budget per size and op")
    p.add_argument("--api", choices=["abi", "codec"], default="abi",
                   help="abi: rs_codec_encode/rs_codec_decode into preallocated buffers "
                        "(the library's rate); codec: the Python Codec mirror (allocates "
                        "per call like the Go codec)")
    args = p.parse_args()

    import numpy as np
    import torch  # noqa: F401  (one HIP runtime; see callfs_amd/_native.py)
    from callfs_amd import Codec, ErasureProfile

    import ctypes
    from callfs_amd import _native as N
    codec = Codec()
    ctx = codec.context
    k, m = args.k, args.m
    prof = ErasureProfile(k, m)
    erase = [int(x) for x in args.erase.split(",") if x]

    def parse(s):
        mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
        return int(s[:-1]) * mult[s[-1]] if s[-1] in mult else int(s)

    for tok in args.sizes.split(","):
        L = parse(tok)
        rng = np.random.default_rng(L)
        objs = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for _ in range(args.threads)]
        enc = [[bytes(s) for s in codec.encode(o, prof)] for o in objs]
        for o, sh in zip(objs, enc):  # correctness of the degraded round trip
            d = [None if i in erase else s for i, s in enumerate(sh)]
            assert codec.decode(d, prof, L) == o

        S = len(enc[0][0])
        n = k + m

        def abi_buffers(t):
            src = np.frombuffer(objs[t], np.uint8)
            shards_out = np.empty(n * S, np.uint8)
            rec = [np.frombuffer(s, np.uint8).copy() for s in enc[t]]
            out = np.empty(L, np.uint8)
            ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rec])
            return src, shards_out, rec, out, ptrs

        bufs = [abi_buffers(t) for t in range(args.threads)]

        def run(op):
            counts = [0] * args.threads
            stop = time.perf_counter() + args.seconds

            def worker(t):
                o, sh = objs[t], enc[t]
                src, shards_out, rec, out, ptrs = bufs[t]
                ss = ctypes.c_size_t(0)
                while time.perf_counter() < stop:
                    if args.api == "codec":
                        if op == "encode":
                            codec.encode(o, prof)
                        else:
                            codec.decode([None if i in erase else s for i, s in enumerate(sh)],
                                         prof, L)
                    elif op == "encode":
                        rc = N.lib.rs_codec_encode(ctx.handle, k, m, src.ctypes.data, L,
                                                   shards_out.ctypes.data, n * S, ctypes.byref(ss))
                        assert rc == 0, rc
                    else:
                        lens = (ctypes.c_size_t * n)(*[0 if i in erase else S for i in range(n)])
                        rc = N.lib.rs_codec_decode(ctx.handle, k, m, ptrs, lens,
                                                   out.ctypes.data, L)
                        assert rc == 0, rc
                    counts[t] += 1

            ths = [threading.Thread(target=worker, args=(t,)) for t in range(args.threads)]
            t0 = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            el = time.perf_counter() - t0
            return sum(counts) * L / el / 2**30, sum(counts)

        e_gib, e_n = run("encode")
        d_gib, d_n = run("decode")
        if args.api == "abi":  # the last ABI results must be the exact inverse
            src, shards_out, rec, out, ptrs = bufs[0]
            assert out.tobytes() == objs[0]
            assert all(shards_out[i * S:(i + 1) * S].tobytes() == enc[0][i] for i in range(n))
        print(json.dumps({"api": args.api, "k": k, "m": m, "object_bytes": L, "threads": args.threads,
                          "erase": erase, "encode_gib_s": round(e_gib, 3),
                          "decode_gib_s": round(d_gib, 3), "encode_calls": e_n,
                          "decode_calls": d_n}), flush=True)


if __name__ == "__main__":
    main()
