"""Seeded object sizes for a rule-vs-tuner sweep at sizes the rule was not fitted on
(development tool). CallFS objects have any size, so shard sizes fall anywhere between the
33 fitted cells; this prints tools/ceiling_sweep.py --shape arguments for encode launches of
the common profiles at log-uniform object sizes (256 KiB - 256 MiB), ~4 GiB batches, planar.
usage: python tools/ceiling_sweep.py --tune 1 --only prod,tuned $(python tools/random_sizes.py [n] [seed])
"""
import sys

import numpy as np

PROFILES = [(4, 2), (6, 3), (8, 4), (10, 4), (12, 4), (16, 4), (8, 8), (10, 8)]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 56
    seed = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0x5112E
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k, m = PROFILES[i % len(PROFILES)]
        L = int(np.exp(rng.uniform(np.log(256 << 10), np.log(256 << 20))))
        S = -(-L // k)
        B = max(1, (4 << 30) // (S * (k + m)))
        out.append(f"--shape {k},{m},{S},{B},-,planar")
    print(" ".join(out))


if __name__ == "__main__":
    main()
