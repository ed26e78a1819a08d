"""Probe: RS kernels reading and writing rs_host_alloc memory directly over PCIe
(development tool, not product).

rs_host_alloc memory is page-locked and mapped into every device's address space at the
same virtual address, so a device plan can take host pointers. This times one plan
launch over host shards (inputs read by the kernel over PCIe, parity written back over
PCIe) against H2D + launch + D2H through device buffers, and checks the bytes against
the CPU oracle.

usage: python tests/perf/zerocopy_probe.py [--k 10 --m 4 --object-bytes 67108864]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from callfs_amd import _native as N  # noqa: E402
from callfs_amd.device import Plan  # noqa: E402
from oracle import cref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--object-bytes", type=int, default=64 << 20)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    k, m = a.k, a.m
    n = k + m
    S = -(-a.object_bytes // k)
    S = (S + 255) // 256 * 256
    ctx = N.default_context()
    buf = N.PinnedBuffer(n * S, ctx)
    buf.array[: k * S] = np.random.default_rng(1).integers(0, 256, k * S, dtype=np.uint8)
    ptrs = [buf.ptr + i * S for i in range(n)]
    plan = Plan(k, m, S, 1, ptrs)
    stream = torch.cuda.current_stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    t_zc = timed(lambda: plan.launch(stream))
    want = cref.encode([buf.array[i * S:(i + 1) * S] for i in range(k)], k, m, simd=True,
                       nthreads=8)
    ok = all(np.array_equal(buf.array[(k + j) * S:(k + j + 1) * S], want[j]) for j in range(m))
    # baseline: H2D of the data, launch on device shards, D2H of the parity
    dev = torch.empty(n * S, dtype=torch.uint8, device="cuda")
    dplan = Plan(k, m, S, 1, [dev.data_ptr() + i * S for i in range(n)])
    host = torch.from_numpy(buf.array).view(torch.uint8)

    def staged():
        dev[: k * S].copy_(host[: k * S], non_blocking=True)
        dplan.launch(stream)
        host[k * S:].copy_(dev[k * S:], non_blocking=True)

    t_st = timed(staged)
    L = k * S
    print(json.dumps({"k": k, "m": m, "object_bytes": L, "zero_copy_ms": round(t_zc, 3),
                      "zero_copy_GiB_s": round(L / (t_zc * 1e-3) / 2**30, 2),
                      "pcie_GB_s": round(n * S / (t_zc * 1e-3) / 1e9, 1),
                      "staged_ms": round(t_st, 3),
                      "staged_GiB_s": round(L / (t_st * 1e-3) / 2**30, 2),
                      "bit_exact": ok}))
    plan.close()
    dplan.close()
    buf.close()


if __name__ == "__main__":
    main()
