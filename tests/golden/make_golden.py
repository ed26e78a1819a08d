"""Generate tests/golden/vectors.json from the CPU oracle (oracle/rs_oracle.py).

The reference (Go + klauspost/reedsolomon v1.13.3) cannot be built or run in this
container (no Go toolchain, module absent, no network — SURVEY.md 8c), so the vectors
come from the oracle, which is itself pinned by the upstream known-answer values
(oracle.rs_oracle.check_kats, run first). Inputs are seeded numpy PCG64 streams, so
the GPU box regenerates identical inputs from (seed, len).

    raw    — small objects: input hex and every shard's hex
    digest — MiB-scale objects: (seed, len) and SHA-256 of every shard
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import rs_oracle as o  # noqa: E402


def rnd(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def main():
    o.check_kats()
    raw = []
    for name, k, m, data in [
        ("hi_rs4_2", 4, 2, b"hi"),
        ("hello_rs2_1", 2, 1, b"hello world"),
        ("tiny_rs10_4", 10, 4, b"0123456789abcdefXYZ"),
        ("4k_rs3_2", 3, 2, rnd(3002, 4096)),
        ("4k_rs10_4", 10, 4, rnd(10004, 4096)),
        ("4k_rs16_4", 16, 4, rnd(16004, 4096)),
        ("4k1_rs5_5", 5, 5, rnd(5005, 4097)),
    ]:
        shards = o.codec_encode(data, k, m)
        raw.append({"name": name, "k": k, "m": m, "data": data.hex(),
                    "shards": [bytes(s).hex() for s in shards]})
    digest = []
    for name, k, m, seed, length in [
        ("1mib_rs3_2", 3, 2, 0xCA11F5, 1 << 20),            # configs[0]
        ("10mib_rs10_4", 10, 4, 0xCA11F5 + 1, 10 << 20),    # north-star shard size
        ("64mib_rs10_4", 10, 4, 0xCA11F5 + 2, 64 << 20),    # configs[1] object size
        ("1mib_rs16_4", 16, 4, 0xCA11F5 + 3, 1 << 20),      # configs[4] sweep point
        ("4kib_rs16_4", 16, 4, 0xCA11F5 + 4, 4 << 10),
    ]:
        shards = o.codec_encode(rnd(seed, length), k, m)
        digest.append({"name": name, "k": k, "m": m, "seed": seed, "len": length,
                       "shard_sha256": [hashlib.sha256(bytes(s)).hexdigest() for s in shards]})
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vectors.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle/rs_oracle.py)",
                   "raw": raw, "digest": digest}, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
