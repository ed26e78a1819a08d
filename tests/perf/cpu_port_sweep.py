"""Per-call encode rate of the CPU port of upstream's SIMD codec (development tool).

Times oracle/rs_oracle.c orc_apply_simd (GFNI, byte ranges on a persistent thread pool,
like upstream codeSomeShardsP) computing the m parity shards of one object per call,
data shards aliasing the object as upstream Split does. Paired with
`CALLFS_E2E_ENCODER=1 tools/e2e_native` (the GPU path the cgo shim takes) it gives the
object size above which the shim should hand a request to the GPU
(CALLFS_ERASURE__GPU_MIN_BYTES).

usage: python tests/perf/cpu_port_sweep.py [--k 10 --m 4 --threads 1,16 --sizes 64K,1M,...]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from oracle import cref  # noqa: E402


def parse_size(s):
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(s[:-1]) * mult[s[-1]] if s[-1] in mult else int(s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--sizes", default="64K,256K,1M,4M,16M,64M")
    ap.add_argument("--seconds", type=float, default=1.0)
    a = ap.parse_args()
    k, m = a.k, a.m
    E = np.zeros((k + m) * k, np.uint8)
    cref.lib().orc_encode_matrix(k, m, E.ctypes.data_as(cref.ctypes.POINTER(cref.ctypes.c_uint8)))
    P = E.reshape(k + m, k)[k:].copy()
    for L in [parse_size(s) for s in a.sizes.split(",")]:
        S = -(-L // k)
        obj = np.random.default_rng(L).integers(0, 256, S * k, dtype=np.uint8)
        data = [obj[i * S:(i + 1) * S] for i in range(k)]
        for th in [int(t) for t in a.threads.split(",")]:
            cref.apply(P, data, simd=True, nthreads=th)
            n, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < a.seconds:
                cref.apply(P, data, simd=True, nthreads=th)
                n += 1
            el = time.perf_counter() - t0
            print(json.dumps({"api": "cpu-port", "k": k, "m": m, "object_bytes": L,
                              "threads": th, "encode_gib_s": round(n * L / el / 2**30, 3),
                              "us_per_call": round(el / n * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
