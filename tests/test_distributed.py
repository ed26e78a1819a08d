"""N>1 path on CPU: world_size-2 gloo process group (127.0.0.1).

Each rank takes its byte-column slice of one object (callfs_amd.sharding, the
configs[3] layout), computes that slice's parity (the CPU oracle stands in for the
per-GPU kernel here: these tests check partitioning, control and reassembly, not the
kernel), and rank 0 reassembles the slices and compares with the whole-object parity.
Also checks the max-over-ranks timer reduction the bench uses."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from callfs_amd.sharding import column_slices, stripe_slices


def test_column_slices_cover_exactly():
    for S in [0, 1, 255, 256, 257, 6_710_887, 107_374_183, 1 << 20]:
        for world in [1, 2, 3, 4, 8]:
            sl = column_slices(S, world)
            assert len(sl) == world
            pos = 0
            for off, w in sl:
                if w:
                    assert off == pos
                pos = off + w if w else pos
            assert sum(w for _, w in sl) == S
            assert all(off % 256 == 0 for off, w in sl if w)


def test_stripe_slices():
    for batch in [1, 7, 256]:
        for world in [1, 2, 8]:
            sl = stripe_slices(batch, world)
            assert sum(c for _, c in sl) == batch
            assert [f for f, _ in sl] == sorted(f for f, _ in sl)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from callfs_amd.sharding import column_slices, max_over_ranks
    from oracle import cref

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k, m, S = 10, 4, 100_003
    rng = np.random.default_rng(2024)  # same object on every rank
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    off, w = column_slices(S, world)[rank]
    par = cref.encode([d[off:off + w] for d in data], k, m) if w else [np.zeros(0, np.uint8)] * m
    mine = torch.from_numpy(np.concatenate(par)) if w else torch.zeros(0, dtype=torch.uint8)
    sizes = [None] * world
    dist.all_gather_object(sizes, (off, w))
    gathered = [None] * world
    dist.all_gather_object(gathered, mine.numpy().tobytes())
    t = max_over_ranks(0.25 * (rank + 1))
    dist.barrier()
    if rank == 0:
        full = cref.encode(data, k, m)
        ok = True
        for (o, ww), blob in zip(sizes, gathered):
            sl = np.frombuffer(blob, np.uint8).reshape(m, ww) if ww else None
            for j in range(m):
                if ww and not np.array_equal(sl[j], full[j][o:o + ww]):
                    ok = False
        q.put((ok, t))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_column_split_reassembles_parity(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ok, t = q.get(timeout=5)
    assert ok
    assert t == pytest.approx(0.25 * world)
