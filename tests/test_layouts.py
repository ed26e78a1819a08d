"""StripeBatch layouts on the CPU (no GPU): every layout's shard pointers, views, gather and
zero_shard address the same bytes, and the readall layout follows upstream Split of an
io.ReadAll body (data shards at pitch S inside one body per object, parity 64-B aligned
at a pitch of S rounded up to 64 B: reedsolomon v1.13.3 Split / AllocAligned)."""
import pytest
import torch

from callfs_amd.device import StripeBatch


@pytest.mark.parametrize("layout", ["pitch", "split", "readall", "planar", "shardmajor"])
@pytest.mark.parametrize("k,m,S,batch", [(10, 4, 1001, 3), (4, 2, 4096, 2), (6, 3, 17, 5)])
def test_layout_views_and_pointers_agree(layout, k, m, S, batch):
    sb = StripeBatch(k, m, S, batch, torch.device("cpu"), layout=layout)
    sb.fill_random(S)
    g = sb.gather()
    assert g.shape == (batch, k + m, S)
    ptrs = sb.pointers()
    for b in range(batch):
        for i in range(k + m):
            t = sb.shard(b, i)
            assert t.data_ptr() == ptrs[b * (k + m) + i], (b, i)
            assert torch.equal(t, g[b, i])
    assert torch.equal(sb.data(), g[:, :k]) and torch.equal(sb.parity(), g[:, k:])
    sb.zero_shard(1)
    sb.zero_shard(k)
    g2 = sb.gather()
    assert int(g2[:, 1].sum()) == 0 and int(g2[:, k].sum()) == 0
    assert torch.equal(g2[:, 2:k], g[:, 2:k])


def test_readall_layout_is_upstream_split_of_a_body():
    k, m, S = 10, 4, 6_710_887 // 1024
    sb = StripeBatch(k, m, S, 3, torch.device("cpu"), layout="readall")
    p = sb.pointers()
    for b in range(3):
        body = p[b * (k + m)]
        assert body % StripeBatch.BODY_ALIGN == 0
        assert [p[b * (k + m) + i] - body for i in range(k)] == [i * S for i in range(k)]
        par = p[b * (k + m) + k:(b + 1) * (k + m)]
        assert all(x % 64 == 0 for x in par)
        assert [y - x for x, y in zip(par, par[1:])] == [-(-S // 64) * 64] * (m - 1)


def test_planar_layout_separates_data_and_parity():
    k, m, S = 10, 4, 1 << 16
    sb = StripeBatch(k, m, S, 4, torch.device("cpu"), layout="planar")
    p = sb.pointers()
    data = sorted(p[b * (k + m) + i] for b in range(4) for i in range(k))
    par = sorted(p[b * (k + m) + k + j] for b in range(4) for j in range(m))
    assert all(x % 256 == 0 for x in data + par)
    assert data[-1] + S <= par[0] or par[-1] + S <= data[0]  # two disjoint regions


@pytest.mark.parametrize("layout", ["planar", "pitch", "shardmajor"])
def test_explicit_pitch(layout):
    """StripeBatch(pitch=P) (bench.py --pitch, tools/jobs.sh pitch_sweep): every shard at that
    pitch within its region; a pitch below S, not a multiple of 16, or for an upstream Split
    layout is refused."""
    k, m, S, P = 10, 4, 6_710_887 // 64, 6_710_887 // 64 + 4096 + 9
    P -= P % 16
    sb = StripeBatch(k, m, S, 3, torch.device("cpu"), layout=layout, pitch=P)
    assert sb.pitch == P
    p = sb.pointers()
    for b in range(3):
        assert [p[b * (k + m) + i + 1] - p[b * (k + m) + i] for i in range(k - 1)] == [
            P if layout != "shardmajor" else 3 * P] * (k - 1)
    sb.fill_random(1)
    assert sb.gather().shape == (3, k + m, S)
    for bad in (S - 16, P + 8):
        with pytest.raises(ValueError):
            StripeBatch(k, m, S, 1, torch.device("cpu"), layout=layout, pitch=bad)
    for split in ("split", "readall"):
        with pytest.raises(ValueError):
            StripeBatch(k, m, S, 1, torch.device("cpu"), layout=split, pitch=P)
