"""Partitioning of RS work across GPUs (one process per GPU, no data-path collective).

Reed-Solomon is column-independent: output byte b of every shard depends only on
byte b of the k input shards (codec.go:36 -> upstream Encode). So work splits with no
exchange step:

* independent stripes (objects) are dealt to ranks (weak scaling: each rank owns its
  batch) — the default bench line;
* one large object (configs[3]: 1 GiB RS(10,4) over 8 GPUs) is split by byte columns:
  rank r owns [off_r, off_r + w_r) of every shard, 256-B aligned except the last, so
  each GPU encodes its slice of all k data shards into the same slice of the m parity
  shards (strong scaling). The union of the slices is the whole object, bit-exact.

The only cross-rank operations are control: a barrier and the max-reduce of the
timer (gloo on CPU tensors).
"""
from __future__ import annotations

from typing import List, Tuple


def column_slices(S: int, world: int, align: int = 256) -> List[Tuple[int, int]]:
    """(offset, width) of each rank's byte columns of an S-byte shard; widths are
    multiples of `align` except the last; every byte is owned by exactly one rank."""
    if world < 1 or S < 0:
        raise ValueError("bad world/S")
    per = -(-S // world)
    per = -(-per // align) * align
    out = []
    for r in range(world):
        off = min(r * per, S)
        out.append((off, max(0, min(per, S - off))))
    return out


def stripe_slices(batch: int, world: int) -> List[Tuple[int, int]]:
    """(first stripe, count) per rank for a fixed total batch (strong scaling)."""
    base, extra = divmod(batch, world)
    out, first = [], 0
    for r in range(world):
        c = base + (1 if r < extra else 0)
        out.append((first, c))
        first += c
    return out


def max_over_ranks(x: float) -> float:
    """Max of a per-rank float over the default process group (identity when none)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])
