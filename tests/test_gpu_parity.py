"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Integer/byte work, so every comparison is bit-exact. Mirrors erasure/codec_test.go
(TestEncodeDecodeRoundtrip 9-35, TestDecodeDegraded 37-63, TestDecodeFailsTooManyMissing
65-88, TestShardChecksum 90-107, TestEncodeInvalidProfile 109-121, TestEncodeSmallData
123-142) and adds known-answer, oracle-parity, erasure-pattern and full-size property
cases.
"""
import json
import os
import threading

import numpy as np
import pytest

from oracle import cref
from oracle import rs_oracle as o

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def codec(native_lib):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from callfs_amd import Codec
    return Codec()


def rnd(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def oracle_shards(data: bytes, k: int, m: int):
    S = (len(data) + k - 1) // k
    buf = np.zeros(S * k, np.uint8)
    buf[: len(data)] = np.frombuffer(data, np.uint8)
    dsh = [buf[i * S:(i + 1) * S] for i in range(k)]
    return dsh + cref.encode(dsh, k, m)


# ---- codec_test.go mirrors ----------------------------------------------------------

def test_encode_decode_roundtrip(codec):
    from callfs_amd import ErasureProfile
    profile = ErasureProfile(data_shards=4, parity_shards=2)
    original = os.urandom(1024 * 100)
    shards = codec.encode(original, profile)
    assert len(shards) == 6
    assert codec.decode(list(shards), profile, len(original)) == original


def test_decode_degraded(codec):
    from callfs_amd import ErasureProfile
    profile = ErasureProfile(4, 2)
    original = os.urandom(1024 * 50)
    shards = list(codec.encode(original, profile))
    shards[1] = None
    shards[4] = None
    assert codec.decode(shards, profile, len(original)) == original
    assert shards[1] is not None and shards[4] is not None  # Decode mutates its shards


def test_decode_fails_too_many_missing(codec):
    from callfs_amd import ErasureProfile, ErasureError, ErrTooFewShards
    profile = ErasureProfile(4, 2)
    original = os.urandom(1024 * 50)
    shards = list(codec.encode(original, profile))
    shards[0] = shards[2] = shards[4] = None
    with pytest.raises(ErasureError) as ei:
        codec.decode(shards, profile, len(original))
    assert isinstance(ei.value, ErrTooFewShards)
    assert str(ei.value) == "erasure: reconstruction failed: too few shards given"


def test_shard_checksum():
    from callfs_amd import shard_checksum
    c = shard_checksum(b"hello world")
    assert len(c) == 64
    assert shard_checksum(b"hello world") == c
    assert shard_checksum(b"hello world!") != c


def test_encode_invalid_profile(codec):
    from callfs_amd import ErasureProfile, ErrInvalidProfile
    with pytest.raises(ErrInvalidProfile):
        codec.encode(b"test", ErasureProfile(0, 2))
    with pytest.raises(ErrInvalidProfile):
        codec.encode(b"test", ErasureProfile(4, 0))


def test_encode_small_data(codec):
    from callfs_amd import ErasureProfile
    profile = ErasureProfile(4, 2)
    shards = codec.encode(b"hi", profile)
    assert [bytes(s) for s in shards] == [b"h", b"i", b"\0", b"\0", b"\x19", b"\x1e"]
    assert codec.decode(list(shards), profile, 2) == b"hi"


# ---- known answers and oracle parity -------------------------------------------------

def test_one_encode_kat(native_lib):
    from callfs_amd import encode_shards
    k, m, data, want = o.KATS["one_encode"]
    shards = [bytearray(d) for d in data] + [bytearray(2) for _ in range(m)]
    encode_shards(shards, k, m)
    assert [list(s) for s in shards[k:]] == want


def test_golden_fixtures(codec):
    from callfs_amd import ErasureProfile
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        vec = json.load(f)
    for case in vec["raw"]:
        data = bytes.fromhex(case["data"])
        shards = codec.encode(data, ErasureProfile(case["k"], case["m"]))
        assert [bytes(s).hex() for s in shards] == case["shards"], case["name"]
    import hashlib
    for case in vec["digest"]:
        data = rnd(case["seed"], case["len"])
        shards = codec.encode(data, ErasureProfile(case["k"], case["m"]))
        got = [hashlib.sha256(bytes(s)).hexdigest() for s in shards]
        assert got == case["shard_sha256"], case["name"]


# R = m rows per launch group: 1..4 take the v_perm kernel, 5..8 the LDS kernel with
# 8-byte nibble entries, 9..16 with 16-byte entries; m > 16 splits (20 = 16+4).
PROFILES = [(1, 1), (2, 1), (3, 2), (2, 3), (3, 4), (4, 2), (5, 5), (6, 3), (8, 4), (10, 4), (12, 4),
            (16, 4), (17, 3), (10, 6), (12, 7), (20, 10), (32, 8), (6, 9), (4, 13),
            (10, 12), (12, 16), (40, 20)]


@pytest.mark.parametrize("k,m", PROFILES)
@pytest.mark.parametrize("L", [1, 15, 16 * 10 + 3, 4096, 65536 + 7, 1 << 20])
def test_encode_matches_oracle(codec, k, m, L):
    from callfs_amd import ErasureProfile
    data = rnd(1000 + k * 31 + m * 7 + L, L)
    got = codec.encode(data, ErasureProfile(k, m))
    want = oracle_shards(data, k, m)
    for i in range(k + m):
        assert bytes(got[i]) == want[i].tobytes(), (k, m, L, i)


ERASURES_10_4 = [(0, 1, 2, 3), (0, 3, 7, 12), (10, 11, 12, 13), (0,), (13,), (4, 9),
                 (1, 5, 11), ()]


@pytest.mark.parametrize("erase", ERASURES_10_4)
@pytest.mark.parametrize("L", [10 * 1024 * 1024, 1_000_003])
def test_decode_rs10_4_erasures(codec, erase, L):
    from callfs_amd import ErasureProfile
    profile = ErasureProfile(10, 4)
    data = rnd(77 + L, L)
    full = [bytes(s) for s in codec.encode(data, profile)]
    shards = [None if i in erase else full[i] for i in range(14)]
    assert codec.decode(shards, profile, L) == data
    for i in erase:
        assert bytes(shards[i]) == full[i]


def test_decode_corrupt_parity_detected(codec):
    from callfs_amd import ErasureProfile, ErrShardCorrupted
    profile = ErasureProfile(10, 4)
    data = rnd(5, 4 << 20)
    full = [bytearray(s) for s in codec.encode(data, profile)]
    full[12][12345] ^= 0x40
    with pytest.raises(ErrShardCorrupted):
        codec.decode(list(full), profile, len(data))
    # one erasure: shard 12 is still an extra present parity and must be re-checked
    sh = list(full)
    sh[3] = None
    with pytest.raises(ErrShardCorrupted):
        codec.decode(sh, profile, len(data))
    # corrupt shard among the first k present: reconstruct uses it, parity 13 catches it
    sh = [bytes(x) for x in codec.encode(data, profile)]
    sh = [bytearray(x) for x in sh]
    sh[2][7] ^= 1
    sh[0] = None
    with pytest.raises(ErrShardCorrupted):
        codec.decode(sh, profile, len(data))


def test_decode_error_precedence(codec):
    from callfs_amd import (ErasureProfile, ErrInsufficientShards, ErrShardNoData,
                            ErrShardSize, ErrTooFewShards)
    p = ErasureProfile(4, 2)
    sh = [bytes(s) for s in codec.encode(b"x" * 100, p)]
    with pytest.raises(ErrInsufficientShards):
        codec.decode(list(sh), p, 101)
    with pytest.raises(ErrShardNoData):
        codec.decode([None] * 6, p, 10)
    bad = list(sh)
    bad[1] = bad[1][:-1]
    with pytest.raises(ErrShardSize):
        codec.decode(bad, p, 100)
    with pytest.raises(ErrTooFewShards):
        codec.decode(sh[:5], p, 100)


def test_decode_insufficient_fills_missing_entries(codec):
    """codec.go:55 Reconstruct fills the nil entries before the join-length check at
    :73 fails, so ErrInsufficientShards leaves them reconstructed (as the Go shim,
    codec_rocm.go, and upstream do); a Verify failure leaves them filled too."""
    from callfs_amd import ErasureProfile, ErrInsufficientShards, ErrShardCorrupted
    p = ErasureProfile(4, 2)
    data = rnd(11, 1000)
    full = [bytes(s) for s in codec.encode(data, p)]
    sh = [None if i in (1, 4) else full[i] for i in range(6)]
    with pytest.raises(ErrInsufficientShards):
        codec.decode(sh, p, 4 * len(full[0]) + 1)
    assert bytes(sh[1]) == full[1] and bytes(sh[4]) == full[4]
    bad = [bytearray(x) for x in full]
    bad[5][3] ^= 1
    sh = [None if i == 0 else bad[i] for i in range(6)]
    with pytest.raises(ErrShardCorrupted):
        codec.decode(sh, p, len(data))
    assert sh[0] is not None and bytes(sh[0]) == full[0]  # rebuilt from shards 1..4


def test_encoder_level_reconstruct_verify(native_lib):
    from callfs_amd import encode_shards, reconstruct, verify
    k, m, S = 10, 4, 333_331
    data = [bytearray(rnd(i, S)) for i in range(k)]
    shards = data + [bytearray(S) for _ in range(m)]
    encode_shards(shards, k, m)
    assert verify(shards, k, m)
    ref = cref.encode([np.frombuffer(bytes(d), np.uint8) for d in data], k, m)
    assert all(bytes(shards[k + j]) == ref[j].tobytes() for j in range(m))
    full = [bytes(s) for s in shards]
    sh = list(shards)
    sh[2] = sh[11] = None
    reconstruct(sh, k, m)
    assert [bytes(s) for s in sh] == full
    sh[11] = bytearray(sh[11])
    sh[11][0] ^= 0xFF
    assert not verify(sh, k, m)


def test_concurrent_encodes_share_one_codec(codec):
    from callfs_amd import ErasureProfile
    profile = ErasureProfile(10, 4)
    errors = []

    def work(seed):
        try:
            for j in range(4):
                data = rnd(seed * 100 + j, 3_000_000 + seed)
                got = codec.encode(data, profile)
                want = oracle_shards(data, 10, 4)
                assert all(bytes(g) == w.tobytes() for g, w in zip(got, want))
                assert codec.decode([None, None] + [bytes(x) for x in got[2:]], profile,
                                    len(data)) == data
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=work, args=(s,)) for s in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


# ---- device-resident plans -----------------------------------------------------------

def _mid(batch, seed):
    """A seeded interior stripe index (checked beside the first and last)."""
    return int(np.random.default_rng(seed).integers(0, batch)) if batch > 2 else 0


def _batch(k, m, S, batch, seed):
    import torch
    from callfs_amd.device import StripeBatch
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"))
    sb.fill_random(seed)
    return sb


@pytest.mark.parametrize("k,m,S,batch", [(10, 4, 1 << 20, 4), (10, 4, 6_710_887, 2),
                                         (16, 4, 256, 64), (3, 2, 349_526, 3),
                                         (24, 12, 4099, 5)])
def test_plan_encode_matches_oracle(native_lib, k, m, S, batch):
    import torch
    from callfs_amd.device import Plan
    sb = _batch(k, m, S, batch, seed=k * 1000 + S)
    plan = Plan.for_batch(sb)
    plan.launch()
    assert not plan.corrupt()
    torch.cuda.synchronize()
    host = sb.buf[:, :, :S].cpu().numpy()
    for b in {0, _mid(batch, S), batch - 1}:
        want = cref.encode([host[b, i] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(host[b, k + j], want[j]), (b, j)
    assert plan.bytes == batch * S * (k + m)


@pytest.mark.parametrize("fill", [0x00, 0xFF])
@pytest.mark.parametrize("k,m,S,batch", [(10, 4, (1 << 20) + 5, 3), (3, 2, 349_526, 2),
                                         (10, 12, 65_541, 2), (20, 8, 4099, 3)])
def test_plan_constant_inputs(native_lib, fill, k, m, S, batch):
    """SURVEY §8(d) sanity inputs: all-zero data encodes to all-zero parity; all-0xFF data
    gives parity row j = 0xFF * XOR_i P[j][i] in every byte (each kernel family: v_perm for
    k <= 3, LDS for R <= 8 and 9..16, ragged tails); then a decode with m erasures from
    the constant shards restores them, and Verify passes."""
    import torch
    from callfs_amd.device import Plan, StripeBatch
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"))
    sb.buf.fill_(fill)
    sb.buf[:, k:].fill_(0x5A)  # parity rows start as garbage
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    host = sb.buf[:, :, :S].cpu().numpy()
    col = [np.full(1, fill, np.uint8) for _ in range(k)]
    want = cref.encode(col, k, m)
    for j in range(m):
        assert (host[:, k + j] == want[j][0]).all(), j
    if fill == 0:
        assert not host[:, k:].any()
    ref = sb.buf.clone()
    erase = list(range(0, k + m, max(1, (k + m) // m)))[:m]
    for i in erase:
        sb.buf[:, i].fill_(0x33)
    present = [i not in erase for i in range(k + m)]
    dec = Plan.for_batch(sb, present=present)
    dec.launch()
    assert not dec.corrupt()
    assert torch.equal(sb.buf[:, :, :S], ref[:, :, :S])


@pytest.mark.parametrize("erase", ERASURES_10_4)
def test_plan_decode_restores_and_verifies(native_lib, erase):
    import torch
    from callfs_amd.device import Plan
    k, m, S, batch = 10, 4, 1 << 20, 8
    sb = _batch(k, m, S, batch, seed=99)
    Plan.for_batch(sb).launch()
    ref = sb.buf.clone()
    for i in erase:
        sb.buf[:, i].zero_()
    present = [i not in erase for i in range(k + m)]
    dec = Plan.for_batch(sb, present=present)
    dec.launch()
    assert not dec.corrupt()
    assert torch.equal(sb.buf[:, :, :S], ref[:, :, :S])
    # corrupt a parity shard outside the first k present: Verify must flag exactly the
    # stripes that were touched
    extra = [i for i in range(k + m) if present[i]][k:]
    if extra:
        sb.buf[3, extra[0], 1000] ^= 1
        sb.buf[6, extra[-1], S - 1] ^= 0x80
        dec.launch()
        assert dec.corrupt_stripes() == [3, 6]
        dec.launch()
        assert dec.corrupt()
        dec.launch()
        assert dec.corrupt_stripes() == [3, 6]


@pytest.mark.parametrize("k,m,S,off", [(10, 4, 100_003, 3), (3, 2, 349_526, 1),
                                       (16, 4, 65_537, 15), (10, 9, 4_099, 7)])
def test_plan_misaligned_pointers(native_lib, k, m, S, off):
    """Shards aliasing one contiguous object (upstream Split layout) at odd S: every shard
    starts at a different byte misalignment; the vector kernels (v_perm for k <= 3, LDS
    otherwise, 16-row group for m = 9) read and write them with unaligned 16-B accesses,
    the byte kernel takes the S % 16 tail. Encode, then a degraded decode, vs the oracle."""
    import torch
    from callfs_amd.device import Plan
    n = k + m
    buf = torch.randint(0, 256, (n * S + 32,), dtype=torch.uint8, device="cuda:0")
    base = buf.data_ptr() + off
    ptrs = [base + i * S for i in range(n)]
    Plan(k, m, S, 1, ptrs).launch()
    torch.cuda.synchronize()
    host = buf.cpu().numpy()[off:off + n * S].copy()
    want = cref.encode([host[i * S:(i + 1) * S] for i in range(k)], k, m)
    for j in range(m):
        assert np.array_equal(host[(k + j) * S:(k + j + 1) * S], want[j]), j
    erase = [0, k - 1, k + m - 1][:m]
    for i in erase:
        buf[off + i * S:off + (i + 1) * S].zero_()
    present = [i not in erase for i in range(n)]
    dec = Plan(k, m, S, 1, ptrs, present=present)
    dec.launch()
    assert not dec.corrupt()
    assert np.array_equal(buf.cpu().numpy()[off:off + n * S], host)


@pytest.mark.parametrize("k,m,S,pitch,batch", [
    (10, 4, (12 << 20) + 1000, 16 << 20, 2),  # addr_tz 24, S <= 32 MiB: 16 column segments
    (6, 3, (20 << 20) + 77, 24 << 20, 1),     # addr_tz 23: 8 column segments
    (10, 4, (40 << 20) + 5, 48 << 20, 1),     # addr_tz 24, S > 32 MiB: 8 segments
    (10, 4, (9 << 20) + 3, (9 << 20) + 256, 2),  # few trailing zeros: consecutive tiles
    (16, 4, 700_000, 1 << 20, 3),             # <= 1 MiB: 2-stripe interleave
    (4, 2, (3 << 20) + 9, 4 << 20, 3),        # 1-8 MiB, 6 streams: consecutive
    (12, 4, 100_000, 1 << 17, 5),             # stripes exactly 2 MiB apart: consecutive
    (4, 4, 120_000, 1 << 17, 6),              # stripes exactly 1 MiB apart: 2-stripe interleave
    (3, 2, (12 << 20) + 100, 16 << 20, 2),    # v_perm kernel (k <= 3), 16 column segments
    (2, 3, 300_001, 300_032, 5),              # v_perm kernel, 2-stripe interleave, odd batch
    (4, 4, 100_000, 1 << 17, 9),              # <= 256 KiB: 8-stripe interleave, ragged group
    (10, 12, (3 << 20) + 4112, 4 << 20, 2),   # 16-row group >= 2 MiB: 8 column segments
    (10, 16, (1 << 20) + 48, 2 << 20, 1),     # 16-row group < 2 MiB: consecutive
    (240, 16, (2 << 20) + 16, (2 << 20) + 256, 1),  # > 64 KiB of LDS tables, segments
])
def test_plan_tile_orders_vs_oracle(native_lib, k, m, S, pitch, batch):
    """Every LDS-kernel tile order of rs_kernels.hip lds_tile_order (keyed on the shard
    size and the power-of-two factor of the shard address differences), with tiles per
    stripe not a multiple of the segment count: encode and a degraded decode, bit-exact
    against the oracle on the first and last stripe."""
    import torch
    from callfs_amd.device import Plan
    n = k + m
    buf = torch.empty(batch * n * pitch, dtype=torch.uint8, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(S)
    buf.random_(0, 256, generator=g)
    ptrs = [buf.data_ptr() + (b * n + i) * pitch for b in range(batch) for i in range(n)]
    Plan(k, m, S, batch, ptrs).launch()
    torch.cuda.synchronize()
    view = buf.view(batch, n, pitch)[:, :, :S]
    want_all = view.cpu().numpy()
    for b in {0, _mid(batch, S), batch - 1}:
        want = cref.encode([want_all[b, i] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(want_all[b, k + j], want[j]), (b, j)
    erase = [0, k // 2, n - 1][:m]
    for i in erase:
        view[:, i].fill_(0x5A)
    dec = Plan(k, m, S, batch, ptrs, present=[i not in erase for i in range(n)])
    dec.launch()
    assert not dec.corrupt()
    assert np.array_equal(view.cpu().numpy(), want_all)


@pytest.mark.parametrize("k,m", [(4, 2), (10, 4)])
def test_shard_files_interop_with_cpu_codec(codec, tmp_path, k, m):
    """shards go to disk as raw bytes under
    .erasure/<hash prefix>/<i> (manager.go:171-184). Files written from the GPU codec's
    shards decode with the CPU oracle, files written from the oracle decode with the GPU
    codec (two shards lost each way), and both sets are byte-identical with matching
    ShardChecksum values."""
    from callfs_amd import ErasureProfile, shard_checksum, shard_layout
    L = (1 << 20) + 17
    data = rnd(4242 + k, L)
    prof = ErasureProfile(k, m)

    def write(shards, sub):
        layout = shard_layout(data, shards)
        for (path, csum), sh in zip(layout, shards):
            f = tmp_path / sub / path
            f.parent.mkdir(parents=True, exist_ok=True)
            f.write_bytes(bytes(sh))
            assert shard_checksum(f.read_bytes()) == csum
        return layout

    def read(layout, sub, lost):
        return [None if i in lost else (tmp_path / sub / p).read_bytes()
                for i, (p, _) in enumerate(layout)]

    gpu_layout = write(codec.encode(data, prof), "gpu")
    cpu_layout = write(o.codec_encode(data, k, m), "cpu")
    assert gpu_layout == cpu_layout  # same paths, same bytes (checksums)
    lost = [1, k + m - 1]
    got = o.codec_decode([None if s is None else np.frombuffer(s, np.uint8).copy()
                          for s in read(gpu_layout, "gpu", lost)], k, m, L)
    assert got == data
    assert codec.decode(read(cpu_layout, "cpu", lost), prof, L) == data


def test_full_size_bench_shape_linearity_and_matrix(native_lib):
    """The bench workload at full size (RS(10,4), 1 MiB shards, 256 stripes) through
    size-independent properties, compared on the device: encode is GF(2)-linear
    (parity(A ^ B) == parity(A) ^ parity(B)), and a stripe whose only nonzero data is
    byte value v in shard i has parity row j equal to mul(P[j][i], v) at every byte, with
    P from the oracle's encode matrix (pinned by the upstream known-answer values)."""
    import torch
    from callfs_amd.device import Plan
    k, m, S, batch = 10, 4, 1 << 20, 256
    a = _batch(k, m, S, batch, seed=101)
    b = _batch(k, m, S, batch, seed=202)
    c = _batch(k, m, S, batch, seed=303)
    c.buf[:, :k] = a.buf[:, :k] ^ b.buf[:, :k]
    for sb in (a, b, c):
        Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    assert torch.equal(c.parity(), a.parity() ^ b.parity())
    del b, c
    # impulses: stripe s carries value v = s + 1 in data shard s % k, zeros elsewhere
    a.buf.zero_()
    vals = torch.arange(1, batch + 1, dtype=torch.int64) % 256
    for s in range(batch):
        a.buf[s, s % k, :S] = int(vals[s])
    Plan.for_batch(a).launch()
    torch.cuda.synchronize()
    P = cref.encode_matrix(k, m)[k:]
    want = torch.tensor([[o.gal_mul(int(P[j][s % k]), int(vals[s])) for j in range(m)]
                         for s in range(batch)], dtype=torch.uint8, device=a.buf.device)
    par = a.parity()
    assert torch.equal(par.amin(dim=2), want) and torch.equal(par.amax(dim=2), want)


@pytest.mark.parametrize("k,m,batch", [(3, 2, 1024), (4, 2, 700)])
def test_sliced_launch_grids_roundtrip(native_lib, k, m, batch):
    """Grids of more than twice ~2 GiB of traffic run as consecutive launch slices
    (rs_kernels.hip slice_tiles): RS(3,2) 1 MiB x 1,024 stripes (v_perm kernel, 131,072
    tiles, 3 slices) and RS(4,2) 1 MiB x 700 (LDS kernel, 89,600 tiles, 3 slices). Every
    stripe must round-trip; first, middle and last stripe against the oracle."""
    import torch
    from callfs_amd.device import Plan
    S = 1 << 20
    sb = _batch(k, m, S, batch, seed=batch + k)
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    for b in (0, batch // 2, batch - 1):
        h = sb.buf[b, :, :S].cpu().numpy()
        want = cref.encode([h[i] for i in range(k)], k, m)
        assert all(np.array_equal(h[k + j], want[j]) for j in range(m)), b
    ref = sb.buf.clone()
    erase = [0, k + m - 1]
    for i in erase:
        sb.buf[:, i, :S].fill_(0x33)
    dec = Plan.for_batch(sb, present=[i not in erase for i in range(k + m)])
    dec.launch()
    assert not dec.corrupt()
    assert torch.equal(sb.buf[:, :, :S], ref[:, :, :S])


def test_full_size_config_rs10_4_64mib_roundtrip(native_lib):
    """configs[1]/[2] at full size: 256 objects of 64 MiB (S = 6,710,887; 22.4 GiB of
    shards in HBM). Encode the batch, erase 4 shards per pattern, decode, require every
    byte back (size-independent round-trip property); stripe 0 checked against the
    oracle."""
    import torch
    from callfs_amd.device import Plan
    k, m, S, batch = 10, 4, 6_710_887, 256
    sb = _batch(k, m, S, batch, seed=64)
    enc = Plan.for_batch(sb)
    enc.launch()
    assert not enc.corrupt()
    host0 = sb.buf[0, :, :S].cpu().numpy()
    want = cref.encode([host0[i] for i in range(k)], k, m)
    assert all(np.array_equal(host0[k + j], want[j]) for j in range(m))
    ref = sb.buf.clone()
    for erase in [(0, 1, 2, 3), (0, 3, 7, 12), (10, 11, 12, 13)]:
        for i in erase:
            sb.buf[:, i, :S].fill_(0xA5)
        dec = Plan.for_batch(sb, present=[i not in erase for i in range(14)])
        dec.launch()
        assert not dec.corrupt()
        assert torch.equal(sb.buf[:, :, :S], ref[:, :, :S]), erase


@pytest.mark.parametrize("erase_n", [9, 12, 16])
def test_decode_wide_erasures(codec, erase_n):
    """9..16 erased shards in one launch group (LDS kernel, 16-byte nibble entries)."""
    from callfs_amd import ErasureProfile
    k, m = 20, 16
    L = 3 * 1024 * 1024 + 5
    data = rnd(erase_n, L)
    full = [bytes(s) for s in codec.encode(data, ErasureProfile(k, m))]
    want = oracle_shards(data, k, m)
    assert all(f == w.tobytes() for f, w in zip(full, want))
    rng = np.random.default_rng(erase_n)
    erase = set(rng.choice(k + m, size=erase_n, replace=False).tolist())
    shards = [None if i in erase else full[i] for i in range(k + m)]
    assert codec.decode(shards, ErasureProfile(k, m), L) == data
    assert all(bytes(shards[i]) == full[i] for i in erase)


@pytest.mark.parametrize("k,m", [(200, 56), (255, 1), (128, 128), (1, 255)])
def test_max_profiles_roundtrip(codec, k, m):
    """k+m = 256 is the largest GF(2^8) profile (upstream switches to Leopard above)."""
    from callfs_amd import ErasureProfile
    L = 256 * 1024 + 13
    data = rnd(k * 1000 + m, L)
    got = codec.encode(data, ErasureProfile(k, m))
    want = oracle_shards(data, k, m)
    assert all(bytes(g) == w.tobytes() for g, w in zip(got, want))
    rng = np.random.default_rng(k + m)
    erase = set(rng.choice(k + m, size=min(m, 9), replace=False).tolist())
    shards = [None if i in erase else bytes(s) for i, s in enumerate(got)]
    assert codec.decode(shards, ErasureProfile(k, m), L) == data


def test_leopard_profiles_unsupported(codec):
    from callfs_amd import ErasureProfile, ErrUnsupportedProfile
    with pytest.raises(ErrUnsupportedProfile):
        codec.encode(b"x" * 1000, ErasureProfile(200, 57))
    with pytest.raises(ErrUnsupportedProfile):
        codec.decode([b"x"] * 257, ErasureProfile(200, 57), 10)


def test_small_objects_concurrent(codec):
    """Small requests of mixed sizes and erasure patterns from 12 threads sharing one
    Codec (lanes of one device, reused slot tables): every result exact, and a
    corrupted request fails alone."""
    from callfs_amd import ErasureProfile, ErrShardCorrupted
    profile = ErasureProfile(10, 4)
    errors = []

    def work(tid):
        try:
            rng = np.random.default_rng(500 + tid)
            for j in range(40):
                L = int(rng.integers(1, 60_000))
                data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
                got = [bytes(s) for s in codec.encode(data, profile)]
                want = oracle_shards(data, 10, 4)
                assert all(g == w.tobytes() for g, w in zip(got, want)), (tid, j, L)
                erase = set(rng.choice(14, size=int(rng.integers(0, 5)), replace=False).tolist())
                shards = [None if i in erase else got[i] for i in range(14)]
                if tid == 3 and j % 5 == 0 and len(erase) < 4:
                    extra = [i for i in range(14) if i not in erase][10:]
                    bad = bytearray(shards[extra[0]])
                    bad[0] ^= 0x55
                    shards[extra[0]] = bytes(bad)
                    with pytest.raises(ErrShardCorrupted):
                        codec.decode(shards, profile, L)
                else:
                    assert codec.decode(shards, profile, L) == data, (tid, j, L, erase)
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ts = [threading.Thread(target=work, args=(t,)) for t in range(12)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:3]


def test_empty_and_zero_length_edges(codec):
    """Split of an empty object fails like upstream (codec.go:31-34 -> ErrShortData);
    Decode with originalSize 0 returns an empty buffer after reconstruct+verify."""
    from callfs_amd import ErasureProfile, ErrShortData
    p = ErasureProfile(4, 2)
    with pytest.raises(ErrShortData) as ei:
        codec.encode(b"", p)
    assert str(ei.value) == ("erasure: failed to split data: not enough data to fill the "
                             "number of requested shards")
    sh = [bytes(s) for s in codec.encode(b"abc", p)]
    assert codec.decode([None] + sh[1:], p, 0) == b""


def test_one_gib_object_roundtrip(native_lib):
    """configs[3] object size: RS(10,4) over a 1 GiB object (S = 107,374,183, a 7-byte
    ragged tail), two objects, encode + worst-case decode, bit-exact on device; the first
    and last 1 MiB of object 0's parity checked against the oracle."""
    import torch
    from callfs_amd.device import Plan
    k, m, S, batch = 10, 4, 107_374_183, 2
    sb = _batch(k, m, S, batch, seed=1 << 30)
    Plan.for_batch(sb).launch()
    ref = sb.buf[:, :, :S].clone()
    for sl in (slice(0, 1 << 20), slice(S - (1 << 20), S)):
        host = sb.buf[0, :, sl].cpu().numpy()
        want = cref.encode([host[i] for i in range(k)], k, m)
        assert all(np.array_equal(host[k + j], want[j]) for j in range(m))
    sb.buf[:, :4, :S].zero_()
    dec = Plan.for_batch(sb, present=[i >= 4 for i in range(14)])
    dec.launch()
    assert not dec.corrupt()
    assert torch.equal(sb.buf[:, :, :S], ref)


# ---- batched host calls (rs_encode_batch / rs_reconstruct_batch) --------------------

@pytest.mark.parametrize("k,m", [(10, 4), (16, 4), (3, 2)])
def test_encode_batch_mixed_sizes_match_oracle(native_lib, k, m):
    """Many stripes per call, several shard sizes (grouped), one empty stripe."""
    from callfs_amd import erasure as E
    from callfs_amd._native import RS_E_NO_DATA, RS_OK
    sizes = [256, 1, 4096, 333, 256, 65536, 0, 4096, 70001] * 7
    stripes = [[rnd(1000 * b + i, S) for i in range(k)] for b, S in enumerate(sizes)]
    parity, status = E.encode_batch(stripes, k, m)
    for b, S in enumerate(sizes):
        if S == 0:
            assert status[b] == RS_E_NO_DATA
            continue
        assert status[b] == RS_OK
        want = cref.encode([np.frombuffer(s, np.uint8) for s in stripes[b]], k, m)
        for j in range(m):
            assert bytes(parity[b][j]) == bytes(want[j]), (b, j)


@pytest.mark.parametrize("k,m,S,B", [(4, 2, 1 << 20, 5),   # 2 stripes per chunk, per-shard DMA
                                     (10, 4, 3 << 20, 3),  # one stripe over several column chunks
                                     (16, 4, 256, 3000)])  # thousands of stripes per chunk
def test_encode_batch_chunk_shapes(native_lib, k, m, S, B):
    from callfs_amd import erasure as E
    rng = np.random.default_rng(S + B)
    stripes = [[rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] for _ in range(B)]
    parity, status = E.encode_batch(stripes, k, m)
    assert status == [0] * B
    for b in range(B):  # every stripe: the 2nd+ stripe of a chunk has its own offsets
        want = cref.encode(stripes[b], k, m)
        for j in range(m):
            assert bytes(parity[b][j]) == bytes(want[j]), (b, j)


@pytest.mark.parametrize("k,m,S,B,erase", [(4, 2, 1 << 20, 5, (0, 5)),      # 2 stripes / chunk
                                           (4, 2, 1 << 20, 5, (1,)),        # + verify rows
                                           (10, 4, 400_000, 7, (2, 3, 11))])
def test_reconstruct_batch_chunk_shapes(native_lib, k, m, S, B, erase):
    """Staged reconstruct with several stripes per chunk and per-run DMA (spitch > 4 MiB):
    every stripe's reconstructed shards and verify flag, not only the first of a chunk."""
    from callfs_amd import erasure as E
    rng = np.random.default_rng(S + B + len(erase))
    full = []
    for _ in range(B):
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        full.append(data + cref.encode(data, k, m))
    stripes = [[None if i in erase else bytearray(x.tobytes()) for i, x in enumerate(f)]
               for f in full]
    status = E.reconstruct_batch(stripes, k, m, verify=True)
    assert status == [0] * B
    for b in range(B):
        for i in range(k + m):
            assert bytes(stripes[b][i]) == full[b][i].tobytes(), (b, i)


def test_reconstruct_batch_mixed_patterns_and_errors(native_lib):
    """Per-stripe erasures, a corrupt stripe, too-few and size-mismatch stripes."""
    from callfs_amd import erasure as E
    from callfs_amd._native import (RS_E_CORRUPT, RS_E_SHARD_SIZE, RS_E_TOO_FEW_SHARDS,
                                    RS_OK)
    k, m = 10, 4
    n = k + m
    patterns = [(), (0,), (0, 1, 2, 3), (0, 3, 7, 12), (10, 11, 12, 13), (5, 13)]
    originals, stripes, expect = [], [], []
    for b in range(48):
        S = (1 << 12) if b % 3 else 100_003
        data = [np.frombuffer(rnd(7 * b + i, S), np.uint8) for i in range(k)]
        full = data + cref.encode(data, k, m)
        originals.append(full)
        st = [bytearray(x.tobytes()) for x in full]
        for i in patterns[b % len(patterns)]:
            st[i] = None
        stripes.append(st)
        expect.append(RS_OK)
    # stripe 7: flip a byte of parity 13, present beyond the first k -> corrupt
    stripes[7] = [bytearray(x.tobytes()) for x in originals[7]]
    stripes[7][0] = None
    stripes[7][13][5] ^= 1
    expect[7] = RS_E_CORRUPT
    # stripe 8: five erasures
    for i in range(5):
        stripes[8][i] = None
    expect[8] = RS_E_TOO_FEW_SHARDS
    # stripe 9: one short shard
    stripes[9] = [bytearray(x.tobytes()) for x in originals[9]]
    stripes[9][4] = stripes[9][4][:-1]
    expect[9] = RS_E_SHARD_SIZE
    status = E.reconstruct_batch(stripes, k, m, verify=True)
    assert status == expect
    for b in range(48):
        if expect[b] != RS_OK:
            continue
        for i in range(n):
            assert bytes(stripes[b][i]) == originals[b][i].tobytes(), (b, i)
    assert stripes[8][0] is None  # failed stripes keep their missing entries


def test_reconstruct_batch_matches_single_calls(native_lib):
    """Batched results equal the per-object rs_reconstruct results (RS(16,4), 4 KiB)."""
    from callfs_amd import erasure as E
    k, m = 16, 4
    stripes, singles = [], []
    for b in range(500):
        data = [np.frombuffer(rnd(31 * b + i, 256), np.uint8) for i in range(k)]
        full = [bytearray(x.tobytes()) for x in data + cref.encode(data, k, m)]
        for i in (b % 20, (b * 7 + 3) % 20):
            full[i] = None
        stripes.append(full)
        singles.append(list(full))
    assert E.reconstruct_batch(stripes, k, m, verify=False) == [0] * 500
    for b in range(0, 500, 37):
        E.reconstruct(singles[b], k, m)
        assert [bytes(x) for x in stripes[b]] == [bytes(x) for x in singles[b]]


# ---- one object split over lanes / devices (CALLFS_RS_SPLIT_*) ----------------------

@pytest.mark.parametrize("ways", [2, 3, 5])
def test_split_object_roundtrip_and_corruption(codec, monkeypatch, ways):
    """Column split of a single object over `ways` lanes: bytes equal the oracle, decode
    restores the object, and a flipped parity byte in one part still reports corruption."""
    from callfs_amd import ErasureProfile, ErrShardCorrupted
    monkeypatch.setenv("CALLFS_RS_SPLIT_MIN_BYTES", str(1 << 20))
    monkeypatch.setenv("CALLFS_RS_SPLIT_WAYS", str(ways))
    k, m = 10, 4
    L = 130_000_017  # S = 13,000,002: ragged, 4 KiB-aligned part boundaries inside
    data = rnd(ways, L)
    shards = codec.encode(data, ErasureProfile(k, m))
    want = oracle_shards(data, k, m)
    for i in range(k, k + m):
        assert bytes(shards[i]) == want[i].tobytes(), i
    got = [bytearray(s) for s in shards]
    for i in (0, 3, 7, 12):
        got[i] = None
    assert codec.decode(got, ErasureProfile(k, m), L) == data
    bad = [bytearray(s) for s in shards]
    bad[1] = None
    bad[13][len(bad[13]) - 5] ^= 0x40  # last part of the columns; parity 13 is checked
    with pytest.raises(ErrShardCorrupted):
        codec.decode(bad, ErasureProfile(k, m), L)


def test_plan_launches_replay_in_a_hip_graph(native_lib):
    """rs_plan_launch only enqueues kernels, so encode -> erase -> decode captures into one
    HIP graph; replays on fresh data (same buffers) give oracle parity and restore the
    erased shards, and a corrupted parity is still flagged through the graph."""
    import torch
    from callfs_amd.device import Plan
    k, m, S, batch = 10, 4, 65_541, 6  # ragged: vector + byte kernels in the graph
    erase = (0, 3, 7)  # 11 present: parity 13 is a verify row
    present = [i not in erase for i in range(k + m)]
    sb = _batch(k, m, S, batch, seed=5)
    enc, dec = Plan.for_batch(sb), Plan.for_batch(sb, present=present)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside capture
        enc.launch(s)
        dec.launch(s)
    torch.cuda.synchronize()
    assert not dec.corrupt(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        enc.launch(s)
        for i in erase:
            sb.buf[:, i, :S].zero_()
        dec.launch(s)
    for seed in (11, 12):
        sb.fill_random(seed)
        torch.cuda.synchronize()
        data = sb.buf[:, :k, :S].clone()
        g.replay()
        torch.cuda.synchronize()
        assert not dec.corrupt(s)
        host = sb.buf[:, :, :S].cpu().numpy()
        assert np.array_equal(host[:, :k], data.cpu().numpy())
        for b in sorted({0, _mid(batch, seed), batch - 1}):
            want = cref.encode([host[b, i] for i in range(k)], k, m)
            for j in range(m):
                assert np.array_equal(host[b, k + j], want[j]), (seed, b, j)
    # a decode-only graph still reports corruption of the verify row
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s):
        dec.launch(s)
    sb.buf[2, 13, 17] ^= 1
    g2.replay()
    torch.cuda.synchronize()
    assert dec.corrupt_stripes(s) == [2]


# ---- randomized dispatch coverage ----------------------------------------------------

def _random_cases(n=48, seed=0xD15):
    """Seeded (k, m, S, batch, misalignment, erasures) draws spanning every dispatch path:
    v_perm (k <= 3), LDS narrow (R <= 8) under each tile order (S <= 512 KiB: 8-stripe
    interleave, 2..8 MiB: 2-stripe, else consecutive), LDS wide (R 9..16, 5-slot ring),
    ragged tails and unaligned shard starts."""
    rng = np.random.default_rng(seed)
    sizes = [1, 15, 16, 17, 4095, 65_536 + 3, 262_144, 524_288 + 16, 1 << 20,
             2 * (1 << 20) + 5, 4 << 20, 8 << 20, (8 << 20) + 4096]
    cases = []
    for c in range(n):
        k = int(rng.choice([1, 2, 3, 4, 5, 10, 16, 20, 32]))
        m = int(rng.choice([1, 2, 3, 4, 6, 8, 9, 12, 16]))
        S = int(sizes[c % len(sizes)])
        cap = (64 << 20) // (2 * (k + m))  # <= 64 MiB of shards per case, >= 2 stripes
        if S > cap:
            S = cap - c % 17
        batch = max(2, min(4, (64 << 20) // (S * (k + m))))
        off = int(rng.integers(0, 16)) if c % 3 == 0 else 0
        ne = int(rng.integers(0, m + 1))
        erase = sorted(rng.choice(k + m, size=ne, replace=False).tolist())
        cases.append((k, m, S, batch, off, erase))
    return cases


@pytest.mark.parametrize("k,m,S,batch,off,erase", _random_cases())
def test_random_plans_vs_oracle(native_lib, k, m, S, batch, off, erase):
    """Device plans over a contiguous [stripe][shard] layout with pitch S + 16 (so a
    nonzero `off` misaligns every shard differently): encode vs the C oracle on the first
    and last stripe, then erase, decode, and require every stripe back bit-exactly with
    no Verify flag."""
    import torch
    from callfs_amd.device import Plan
    n = k + m
    pitch = S + 16
    buf = torch.randint(0, 256, (batch * n * pitch + 16,), dtype=torch.uint8, device="cuda:0")
    base = buf.data_ptr() + off
    ptrs = [base + (b * n + i) * pitch for b in range(batch) for i in range(n)]
    enc = Plan(k, m, S, batch, ptrs)
    enc.launch()
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    view = lambda b, i: host[off + (b * n + i) * pitch: off + (b * n + i) * pitch + S]
    for b in {0, _mid(batch, S), batch - 1}:
        want = cref.encode([view(b, i).copy() for i in range(k)], k, m, simd=True, nthreads=4)
        for j in range(m):
            assert np.array_equal(view(b, k + j), want[j]), (b, j)
    ref = torch.from_numpy(host.copy()).to("cuda:0")
    for b in range(batch):
        for i in erase:
            s0 = off + (b * n + i) * pitch
            buf[s0:s0 + S].zero_()
    dec = Plan(k, m, S, batch, ptrs, present=[i not in erase for i in range(n)])
    dec.launch()
    assert dec.corrupt_stripes() == []
    assert torch.equal(buf, ref)


def _random_layout_cases(n=36, seed=0x5A17):
    """Seeded (layout, k, m, S, batch, erasures, fresh) draws over the layouts the round-5
    rules were fitted on: planar (256-B pitch), readall (upstream Split of an io.ReadAll
    body: odd S puts every data shard at its own offset) and split (pitch S, odd base), with
    shard sizes spanning each rule band (<= 256 KiB, to 1 MiB, the 1-2 MiB Q8 band, above)."""
    rng = np.random.default_rng(seed)
    sizes = [4_097, 87_382, 104_858 + 1, 262_144, 699_051, 1_398_102, 1_677_722 + 1,
             2_097_152, 2_796_203, 4_194_304 + 48]
    cases = []
    for c in range(n):
        layout = ("planar", "readall", "split")[c % 3]
        k = int(rng.choice([4, 6, 8, 10, 12, 16, 20]))
        m = int(rng.choice([2, 3, 4, 8]))
        S = int(sizes[int(rng.integers(0, len(sizes)))])
        batch = max(2, min(4, (48 << 20) // (S * (k + m))))
        ne = int(rng.integers(1, m + 1))
        erase = sorted(rng.choice(k + m, size=ne, replace=False).tolist())
        cases.append((layout, k, m, S, batch, erase, bool(c % 2)))
    return cases


@pytest.mark.parametrize("layout,k,m,S,batch,erase,fresh", _random_layout_cases())
def test_random_layouts_vs_oracle(native_lib, layout, k, m, S, batch, erase, fresh):
    """Plans on the rules alone (untuned) over seeded shapes in the planar, readall and
    split layouts: encode against the C oracle on the first and last stripe, then the
    erased shards rebuilt in place or (fresh) into buffers of their own, every byte back."""
    import torch
    from callfs_amd.device import Plan, StripeBatch, _aligned_empty
    n = k + m
    dev = torch.device("cuda:0")
    sb = StripeBatch(k, m, S, batch, dev, layout=layout)
    sb.fill_random(S ^ (k << 8) ^ m)
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    host = sb.gather().cpu().numpy()
    for b in {0, batch - 1}:
        want = cref.encode([host[b, i].copy() for i in range(k)], k, m, simd=True, nthreads=4)
        for j in range(m):
            assert np.array_equal(host[b, k + j], want[j]), (b, j)
    present = [i not in erase for i in range(n)]
    if fresh:
        out = _aligned_empty((batch, len(erase), -(-S // 64) * 64), 256, dev)
        out.fill_(0x5A)
        ptrs = list(sb.pointers())
        for b in range(batch):
            for j, i in enumerate(erase):
                ptrs[b * n + i] = out[b, j].data_ptr()
        dec = Plan(k, m, S, batch, ptrs, present=present)
    else:
        for i in erase:
            sb.zero_shard(i)
        dec = Plan.for_batch(sb, present=present)
    dec.launch()
    assert dec.corrupt_stripes() == []
    if fresh:
        got = out.cpu().numpy()
        for b in range(batch):
            for j, i in enumerate(erase):
                assert np.array_equal(got[b, j, :S], host[b, i]), (b, i)
    else:
        assert np.array_equal(sb.gather().cpu().numpy(), host)


# ---- zero-copy staging: caller buffers in rs_host_alloc memory -----------------------

def _pinned(n):
    from callfs_amd import _native as N
    return N.PinnedBuffer(n, N.default_context())


@pytest.mark.parametrize("k,m,L", [(10, 4, (64 << 20) + 3), (16, 4, 5_000_000),
                                   (3, 2, 1_048_576), (10, 9, 3_000_001)])
def test_pinned_encode_and_decode_direct(native_lib, k, m, L):
    """Object and shards in rs_host_alloc memory: rs_codec_encode, rs_encode and
    rs_codec_decode (erasures + join into a pinned `out`) take the direct-DMA path; bytes
    equal the oracle, and corruption is still reported."""
    import ctypes
    from callfs_amd import _native as N
    ctx = N.default_context()
    n = k + m
    S = -(-L // k)
    data = np.frombuffer(rnd(L, L), np.uint8)
    src = _pinned(L)
    src.array[:] = data
    sh = _pinned(n * S)
    ss = ctypes.c_size_t()
    N.check(N.lib.rs_codec_encode(ctx.handle, k, m, src.ptr, L, sh.ptr, n * S, ctypes.byref(ss)))
    assert ss.value == S
    want = oracle_shards(data.tobytes(), k, m)
    for i in range(n):
        assert np.array_equal(sh.array[i * S:(i + 1) * S], want[i]), i
    # rs_encode with data aliasing the pinned object (Split layout) and pinned parity
    full = L // S
    par = _pinned(m * S)
    tail = _pinned(max(1, (k - full) * S))  # shards at and after the object's end
    tail.array[:] = 0
    tail.array[:L - full * S] = data[full * S:]
    dptr = [src.ptr + i * S for i in range(full)] + [tail.ptr + i * S for i in range(k - full)]
    N.check(N.lib.rs_encode(ctx.handle, k, m, S, (ctypes.c_void_p * k)(*dptr),
                            (ctypes.c_void_p * m)(*[par.ptr + j * S for j in range(m)])))
    for j in range(m):
        assert np.array_equal(par.array[j * S:(j + 1) * S], want[k + j]), j
    # decode: erase, reconstruct + verify + join into a pinned out
    erase = [0, k - 1, n - 1][:m]
    for i in erase:
        sh.array[i * S:(i + 1) * S] = 0
    lens = (ctypes.c_size_t * n)(*[0 if i in erase else S for i in range(n)])
    ptrs = (ctypes.c_void_p * n)(*[sh.ptr + i * S for i in range(n)])
    out = _pinned(L)
    N.check(N.lib.rs_codec_decode(ctx.handle, k, m, ptrs, lens, out.ptr, L))
    assert np.array_equal(out.array, data)
    for i in erase:
        assert np.array_equal(sh.array[i * S:(i + 1) * S], want[i]), i
    # a flipped byte in a present parity beyond the first k is still caught
    if m > 1:
        sh.array[(n - 1) * S + 17] ^= 0x20
        lens = (ctypes.c_size_t * n)(*[S] * n)
        lens[1] = 0
        assert N.lib.rs_codec_decode(ctx.handle, k, m, ptrs, lens, out.ptr, L) == N.RS_E_CORRUPT
    for b in (src, sh, par, tail, out):
        b.close()


def test_pinned_buffers_reused_with_new_contents(native_lib):
    """The server refills the same pinned buffers for every request: five encodes of
    different data through the same buffers must each match the oracle (no stale lines
    of an earlier call's bytes in device caches)."""
    import ctypes
    from callfs_amd import _native as N
    ctx = N.default_context()
    k, m, S = 10, 4, 1 << 20
    src = _pinned(k * S)
    par = _pinned(m * S)
    dp = (ctypes.c_void_p * k)(*[src.ptr + i * S for i in range(k)])
    pp = (ctypes.c_void_p * m)(*[par.ptr + j * S for j in range(m)])
    for it in range(5):
        src.array[:] = np.frombuffer(rnd(500 + it, k * S), np.uint8)
        N.check(N.lib.rs_encode(ctx.handle, k, m, S, dp, pp))
        want = cref.encode([src.array[i * S:(i + 1) * S] for i in range(k)], k, m, simd=True,
                           nthreads=4)
        for j in range(m):
            assert np.array_equal(par.array[j * S:(j + 1) * S], want[j]), (it, j)
    src.close()
    par.close()


def test_pinned_mixed_with_pageable_uses_staging(native_lib):
    """One pageable output among pinned inputs: the call stays on the staging path and is
    still bit-exact; freeing a pointer rs_host_alloc did not return is RS_E_ARG."""
    import ctypes
    from callfs_amd import _native as N
    ctx = N.default_context()
    k, m, S = 10, 4, 3 << 20
    src = _pinned(k * S)
    src.array[:] = np.frombuffer(rnd(9, k * S), np.uint8)
    par = [bytearray(S) for _ in range(m)]
    par_ptrs = [np.frombuffer(p, np.uint8).ctypes.data for p in par]
    N.check(N.lib.rs_encode(ctx.handle, k, m, S,
                            (ctypes.c_void_p * k)(*[src.ptr + i * S for i in range(k)]),
                            (ctypes.c_void_p * m)(*par_ptrs)))
    want = cref.encode([src.array[i * S:(i + 1) * S] for i in range(k)], k, m, simd=True,
                       nthreads=4)
    for j in range(m):
        assert np.array_equal(np.frombuffer(par[j], np.uint8), want[j])
    assert N.lib.rs_host_free(ctx.handle, ctypes.c_void_p(src.ptr + 1)) == N.RS_E_ARG
    src.close()


# ---- configs[3]: per-rank byte-column slices of 1 GiB objects -------------------------

@pytest.mark.parametrize("world", [8, 3])
def test_configs3_rank_column_slices_reassemble(native_lib, world):
    """BASELINE configs[3] as bench.py --object-bytes runs it on `world` GPUs, every rank
    here on cuda:0: rank r holds columns column_slices(S, world)[r] of all k data shards of
    a 1 GiB RS(10,4) object (S = 107,374,183) in its own StripeBatch, encodes, then decodes
    erase {0,1,2,3} through Plan. The slices reassembled are the whole object's parity and
    reconstruction: compared with the C oracle over the full 1 GiB (16 threads)."""
    import torch
    from callfs_amd.device import Plan, StripeBatch
    from callfs_amd.sharding import column_slices
    k, m, S = 10, 4, 107_374_183
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0F3)
    data = torch.randint(0, 256, (k, S), dtype=torch.uint8, device=dev, generator=g)
    parity = torch.empty((m, S), dtype=torch.uint8, device=dev)
    present = [i not in (0, 1, 2, 3) for i in range(k + m)]
    for off, w in column_slices(S, world):
        if not w:
            continue
        sb = StripeBatch(k, m, w, 1, dev)
        sb.buf[0, :k, :w].copy_(data[:, off:off + w])
        Plan.for_batch(sb).launch()
        parity[:, off:off + w].copy_(sb.buf[0, k:, :w])
        keep = sb.buf[0, :4, :w].clone()
        sb.buf[0, :4, :w].zero_()
        dec = Plan.for_batch(sb, present=present)
        dec.launch()
        assert not dec.corrupt()
        assert torch.equal(sb.buf[0, :4, :w], keep), (off, w)
        del sb, keep
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    want = cref.encode([host[i] for i in range(k)], k, m, simd=True, nthreads=16)
    got = parity.cpu().numpy()
    for j in range(m):
        assert np.array_equal(got[j], want[j]), j


def test_host_pool_reuses_freed_buffers(native_lib):
    """rs_host_free parks a buffer and rs_host_alloc of a similar size gets it back (no new
    page-locking per request); a parked pointer is no longer a valid rs_host_free argument;
    a request much smaller than any parked buffer gets a new one; and a reused buffer with
    stale contents still takes the zero-copy path correctly."""
    import ctypes
    from callfs_amd import _native as N
    ctx = N.Context()
    try:
        k, m, S = 4, 2, 3 << 20
        a = N.PinnedBuffer(k * S, ctx)
        pa = a.ptr
        a.array[:] = 0xEE
        a.close()
        assert N.lib.rs_host_free(ctx.handle, ctypes.c_void_p(pa)) == N.RS_E_ARG  # parked
        b = N.PinnedBuffer(k * S - 4096, ctx)  # within a quarter: the parked buffer
        assert b.ptr == pa
        small = N.PinnedBuffer(4096, ctx)
        assert small.ptr != pa  # pa is in use
        # small requests are matched in 2 MiB allocation granules: alloc/free/alloc of
        # 4 KiB, and then of 1 MiB, gets the same buffer back
        ps = small.ptr
        small.close()
        small = N.PinnedBuffer(4096, ctx)
        assert small.ptr == ps
        small.close()
        mib = N.PinnedBuffer(1 << 20, ctx)
        assert mib.ptr == ps
        mib.close()
        mib = N.PinnedBuffer(1 << 20, ctx)
        assert mib.ptr == ps
        mib.close()
        small = N.PinnedBuffer(4096, ctx)
        par = N.PinnedBuffer(m * S, ctx)
        data = np.frombuffer(rnd(77, k * S), np.uint8)
        b.array[: k * S - 4096] = data[: k * S - 4096]
        view = np.ctypeslib.as_array((ctypes.c_uint8 * (k * S)).from_address(b.ptr))
        view[k * S - 4096:] = data[k * S - 4096:]  # the rest of the reused 2 MiB granule
        dp = (ctypes.c_void_p * k)(*[b.ptr + i * S for i in range(k)])
        pp = (ctypes.c_void_p * m)(*[par.ptr + j * S for j in range(m)])
        N.check(N.lib.rs_encode(ctx.handle, k, m, S, dp, pp))
        want = cref.encode([data[i * S:(i + 1) * S] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(par.array[j * S:(j + 1) * S], want[j]), j
        for buf in (b, small, par):
            buf.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("k,m,S,batch,off", [
    (10, 4, 17, 3, 1),                 # one vector per shard
    (10, 4, 16 * 63 + 5, 4, 7),        # exactly one realigning wave's 63 vectors + tail
    (10, 4, 16 * 64 + 9, 3, 2),        # 64 vectors: the second wave holds one
    (12, 8, 4096 * 3 + 1, 5, 13),      # R = 8, odd stripe stride
    (8, 2, 16 * 504 * 2 + 15, 2, 5),   # k = 8 (the rule's minimum), 504-vector tile boundaries
    (10, 4, 1_000_003, 2, 11),         # Split layout of ~10 MB objects
    # aligned parity stores (REALIGN 2: 62 stored vectors per wave, 496 per tile, edge
    # bytes written by each stripe's first tile)
    (10, 4, 32, 3, 9),                 # two vectors: one aligned block per row at most
    (10, 4, 16 * 62 + 3, 3, 5),        # one wave's 62 stored vectors
    (10, 4, 16 * 63 + 15, 2, 1),       # 63: the second wave stores the last block
    (9, 6, 16 * 496 + 16 * 62 + 1, 2, 14),  # tile and wave boundaries, R = 6
    (10, 4, 16 * 1000, 2, 3),          # S % 16 == 0, every shard misaligned by 3
    (8, 3, 16 * 496 * 3 + 7, 2, 8),    # R = 3, three tiles
])
@pytest.mark.parametrize("form", ["rule", "realign-x32", "realign-tri-x32", "realign-tri"])
def test_plan_misaligned_batch_realign(native_lib, k, m, S, batch, off, form):
    """Contiguous stripes in the upstream Split layout at odd S (every input shard at its
    own byte misalignment, odd stripe stride): k >= 8 launches take the realigning LDS
    kernel (aligned loads, DPP + v_alignbyte), and with misaligned parity rows its form
    that also aligns the stores (62 vectors per wave, edge bytes in the first tile). Encode,
    a decode erasing m shards, and a decode with Verify rows, against the oracle per
    stripe, every byte of every stripe. `form` pins the realigning kernel's ring-of-three
    or triple-load instance (rs_plan_set_orders) instead of the rule's."""
    import torch
    from callfs_amd.device import Plan
    n = k + m
    total = batch * n * S
    buf = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device="cuda:0")
    base = buf.data_ptr() + off
    ptrs = [base + (b * n + i) * S for b in range(batch) for i in range(n)]

    def pinned(plan):
        if form != "rule":
            plan.set_orders([form] * int(N.lib.rs_plan_groups(plan.handle)))
        return plan

    from callfs_amd import _native as N
    pinned(Plan(k, m, S, batch, ptrs)).launch()
    torch.cuda.synchronize()
    host = buf.cpu().numpy()[off:off + total].copy()
    for b in range(batch):
        st = host[b * n * S:(b + 1) * n * S]
        want = cref.encode([st[i * S:(i + 1) * S] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(st[(k + j) * S:(k + j + 1) * S], want[j]), (b, j)
    for erase in (list(range(0, k, max(1, k // m)))[:m], [1, k]):  # m erasures / verify rows
        for b in range(batch):
            for i in erase:
                s0 = off + (b * n + i) * S
                buf[s0:s0 + S].zero_()
        dec = pinned(Plan(k, m, S, batch, ptrs, present=[i not in erase for i in range(n)]))
        dec.launch()
        assert not dec.corrupt(), erase
        assert np.array_equal(buf.cpu().numpy()[off:off + total], host), erase


# ---- tile-order tuning (rs_plan_tune) ----------------------------------------------------

@pytest.mark.parametrize("k,m,S,batch,erase", [
    (10, 4, 1 << 20, 6, None),          # LDS kernel, rule G2: consecutive / G2 timed
    (10, 4, 1 << 20, 6, (0, 3, 7)),     # decode with a Verify row
    (3, 2, 349_526, 8, None),           # v_perm kernel
    (10, 16, 262_144 + 5, 3, None),     # wide group (SDWA addresses), ragged tail
    (20, 20, 65_536, 4, None),          # two launch groups (16 + 4 rows)
    (4, 2, 96, 40, None),               # one tile per stripe: G8 among the candidates
])
def test_plan_tune_then_launch_bit_exact(native_lib, k, m, S, batch, erase):
    """rs_plan_tune launches every candidate order (the outputs are recomputed to the same
    bytes) and later launches use the chosen one: parity / reconstruction stay bit-exact
    against the oracle, and Verify does not flag clean stripes."""
    import torch
    from callfs_amd.device import Plan
    sb = _batch(k, m, S, batch, seed=S + k)
    enc = Plan.for_batch(sb)
    names = enc.tune(reps=1)
    assert len(names) == max(1, -(-m // 16))
    plain = {"consecutive", "g8", "g2", "q8", "q16", "x8", "x32"}
    tri = {"tri", "tri-g2", "tri-x32", "tri-q8", "tri-q16", "tri-x8"}
    # every group may also take its bit-sliced kernel, in any tile order
    plain |= {"bs", "bs-g8", "bs-g2", "bs-q8", "bs-q16", "bs-x8", "bs-x32"}
    # a launch group with R <= 8 rows may also take the triple loads: up to 16 inputs, or
    # any count at R <= 4 (the double-buffered form); groups of 9..16 rows never do
    for gi, name in enumerate(names):
        rows = min(16, m - 16 * gi)
        tri_ok = rows <= 8 and k >= 3 and (k <= 16 or rows <= 4)
        assert name in (plain | tri if tri_ok else plain), (gi, names)
    sb.fill_random(S + k + 1)  # fresh data: the tuned plan must compute it, not reuse
    enc.launch()
    torch.cuda.synchronize()
    host = sb.buf[:, :, :S].cpu().numpy()
    for b in sorted({0, _mid(batch, S), batch - 1}):
        want = cref.encode([host[b, i] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(host[b, k + j], want[j]), (b, j)
    if erase is None:
        return
    ref = sb.buf.clone()
    present = [i not in erase for i in range(k + m)]
    dec = Plan.for_batch(sb, present=present)
    for i in erase:
        sb.buf[:, i].zero_()
    dec.tune(reps=2)
    assert not dec.corrupt()
    for i in erase:
        sb.buf[:, i].zero_()
    dec.launch()
    assert not dec.corrupt()
    assert torch.equal(sb.buf[:, :, :S], ref[:, :, :S])
    sb.buf[1, 13, 77] ^= 4  # parity 13 is a Verify row of this pattern
    dec.launch()
    assert dec.corrupt_stripes() == [1]


ALL_ORDER_NAMES = ["consecutive", "g8", "g2", "q8", "q16", "x8", "x32", "realign",
                   "realign-x8", "realign-x32", "wix", "wix-g8", "wix-g2", "wix-q8", "wix-q16",
                   "wix-x8", "wix-x32", "tri", "tri-g2", "tri-x32", "tri-q8", "tri-q16",
                   "tri-x8", "realign-tri", "realign-tri-x8", "realign-tri-x32",
                   "dma", "dma-g2", "dma-q8", "dma-x32", "tridb-g4", "tridb-g8",
                   "bs", "bs-g8", "bs-g2", "bs-q8", "bs-q16", "bs-x8", "bs-x32"]


@pytest.mark.parametrize("k,m,S,batch,off,erase", [
    (10, 4, (1 << 20) + 16, 3, 0, None),   # aligned: 129 tiles per stripe, X8/X32 groups + tail
    (10, 4, (1 << 20) + 1, 3, 1, None),    # Split layout (odd S): realigning kernel per order
    (10, 4, (1 << 20) + 1, 3, 1, (5,)),    # one erasure: 1 written + 3 Verify rows
    (6, 3, (1 << 18) + 32, 3, 0, (2,)),    # aligned, 1 written + 2 Verify rows (WIX too)
    (10, 8, 300_001, 5, 3, None),          # R = 8, realigning kernel
    (4, 2, 8 * 512 * 16 * 9 + 7, 2, 0, (0, 1)),  # k = 4, R = 2 decode, ragged tail
    (4, 2, (8 << 20) + 8192 * 3 + 16, 2, 0, None),  # > 1024 tiles per stripe: Q8 / Q16
    (5, 3, (8 << 20) + 1, 2, 1, None),     # Split layout, K = 5: realigning triple + 2
    # R 5..8 with Verify rows and K below the A/B build's LDS-DMA ring depth (6): its prefill
    # issues K DMAs and the tail waits vmcnt(K-1-i); ragged S leaves the last tile partial
    # (inactive lanes skip their DMA) -- checked when CALLFS_RS_LIB names the A/B build
    (3, 6, 300_001 - 1, 3, 0, (0,)),
    (5, 7, 8192 * 3 + 16 * 5, 2, 0, (1,)),
    (2, 8, 65_536 + 48, 3, 0, (9,)),
])
def test_plan_every_offered_order_bit_exact(native_lib, k, m, S, batch, off, erase):
    """rs_plan_set_orders pins each tile order the launch group's kernel offers (the
    rs_plan_tune candidates, X8 / X32 and the realigning kernel's orders included); every
    instance recomputes every byte of every stripe as the oracle does, Verify rows pass on
    clean stripes and flag a flipped byte. An order the kernel does not offer is refused
    (RS_E_ARG) and leaves the plan as it was."""
    import torch
    from callfs_amd import _native as N
    from callfs_amd.device import Plan
    n = k + m
    total = batch * n * S
    buf = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device="cuda:0")
    base = buf.data_ptr() + off
    ptrs = [base + (b * n + i) * S for b in range(batch) for i in range(n)]
    host = buf.cpu().numpy()[off:off + total].copy()
    for b in range(batch):  # consistent stripes: oracle parity in place
        st = host[b * n * S:(b + 1) * n * S]
        want = cref.encode([st[i * S:(i + 1) * S] for i in range(k)], k, m)
        for j in range(m):
            st[(k + j) * S:(k + j + 1) * S] = want[j]
    good = torch.from_numpy(host).to("cuda:0")
    present = None if erase is None else [i not in erase for i in range(n)]
    plan = Plan(k, m, S, batch, ptrs, present=present)
    taken = []
    for name in ALL_ORDER_NAMES:
        try:
            plan.set_orders([name])
        except N.NativeError as e:
            assert e.code == N.RS_E_ARG
            continue
        taken.append(name)
        buf[off:off + total].copy_(good)
        for i in (range(k, n) if erase is None else erase):
            for b in range(batch):
                s0 = off + (b * n + i) * S
                buf[s0:s0 + S].zero_()
        plan.launch()
        assert not plan.corrupt(), name
        assert torch.equal(buf[off:off + total], good), name
        if erase is not None and (n - len(erase)) > k:  # a Verify row exists: flip in it
            vrow = max(i for i in range(n) if i not in erase)
            buf[off + (1 * n + vrow) * S + S // 2] ^= 0x40
            plan.launch()
            assert plan.corrupt_stripes() == [1], name
    assert "consecutive" in taken or "realign" in taken, taken
    if (off | S) % 2:  # shards at odd offsets
        assert {"realign", "realign-x8", "realign-x32", "realign-tri", "realign-tri-x8",
                "realign-tri-x32"} <= set(taken), taken
    else:
        if S // 8192 > 1024 and m <= 8:  # tiles per stripe: triple loads in segment orders
            assert {"tri-q8", "tri-q16"} <= set(taken), taken
        assert {"x8", "x32"} <= set(taken), taken
        with pytest.raises(N.NativeError):
            plan.set_orders(["realign"])  # aligned shards: no realigning kernel
    # the 6-bit triple lookups (Policy::WIX 1) and the LDS-DMA ring are A/B-build forms: the
    # product refuses them (run with CALLFS_RS_LIB=callfs_amd/libcallfs_rs_ab.so, the A/B
    # build offers and checks them here)
    if "libcallfs_rs_ab" not in N.LIB_PATH:
        assert not any(t.startswith(("wix", "dma", "tridb-")) for t in taken), taken
    with pytest.raises(N.NativeError):
        plan.set_orders(["none"] * (plan_groups := int(N.lib.rs_plan_groups(plan.handle))) + ["none"])
    plan.set_orders(["none"] * plan_groups)


@pytest.mark.parametrize("k,m,S,erase", [
    (4, 2, (1 << 20) + 16, None),        # CallFS default profile, encode: rule = triples
    (8, 8, 262_144 + 5, None),           # R = 8 (8-byte entries), ragged tail
    (6, 6, 65_536, None),                # 1 MiB-object-sized shards (G8 -> X32)
    (10, 8, 300_000, None),
    (10, 4, 1 << 20, (0, 1, 2, 3)),      # the bench decode
    (4, 2, 1 << 20, ()),                 # download Verify, nothing erased: read-only
    (10, 4, 100_000 + 3, ()),            # read-only, ragged tail compared too
    (5, 3, 1 << 18, (1,)),               # written + Verify rows: triples with early compares (G2)
    (4, 2, (8 << 20) + 16, None),        # K <= 5 above 2 MiB: X32 (round 4)
    (6, 3, (4 << 20) + 32, None),        # K = 6 above 2 MiB: Q16
    (4, 2, (4 << 20) + 7, (1,)),         # K <= 4, written + Verify rows: X32, early compares
    (10, 4, 1 << 20, (5,)),              # one-erasure decode of the bench shape: G2
    (6, 3, (16 << 20) + 48, ()),         # read-only above 2 MiB: X32
    (32, 8, 32_768, None),               # R 5..8 up to 256 KiB: rotating triples at any K
    (16, 8, 65_536 + 9, None),           # ... with a ragged tail
])
def test_plan_rule_triples_vs_oracle(native_lib, k, m, S, erase):
    """The rule's triple-load kernel (tile_order.hpp tri_rule_order: 4 <= K <= 12, R <= 8;
    launches that write every row or compare every row, and R <= 4 launches with written
    and Verify rows through the early-compare form): encode / reconstruct every byte of
    every stripe as the oracle does; launches with Verify rows pass clean stripes and flag
    exactly the stripe with a flipped byte, also in the ragged tail."""
    import torch
    from callfs_amd.device import Plan
    n, batch = k + m, 3
    pitch = (S + 255) // 256 * 256
    buf = torch.randint(0, 256, (batch, n, pitch), dtype=torch.uint8, device="cuda:0")
    ptrs = [buf[b, i].data_ptr() for b in range(batch) for i in range(n)]
    Plan(k, m, S, batch, ptrs).launch()
    torch.cuda.synchronize()
    h = buf.cpu().numpy()
    for b in range(batch):
        want = cref.encode([h[b, i, :S] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(h[b, k + j, :S], want[j]), (b, j)
    if erase is None:
        return
    good = buf.clone()
    dec = Plan(k, m, S, batch, ptrs, present=[i not in erase for i in range(n)])
    for i in erase:
        buf[:, i].zero_()
    dec.launch()
    assert not dec.corrupt()
    assert torch.equal(buf[:, :, :S], good[:, :, :S])
    if len(erase) < m:  # a Verify row exists
        row = n - 1
        buf[2, row, S - 1] ^= 0x01  # last byte: the ragged tail when S % 16 != 0
        dec.launch()
        assert dec.corrupt_stripes() == [2]


def test_plan_tune_argument_errors(native_lib):
    import ctypes
    from callfs_amd import _native as N
    from callfs_amd.device import Plan
    sb = _batch(4, 2, 4096, 2, seed=3)
    p = Plan.for_batch(sb)
    assert N.lib.rs_plan_tune(p.handle, None, 0, None, 0) == N.RS_E_ARG        # reps < 1
    assert N.lib.rs_plan_tune(p.handle, None, 1, None, 2) == N.RS_E_ARG        # no array
    assert N.lib.rs_plan_tune(None, None, 1, None, 0) == N.RS_E_ARG
    out = (ctypes.c_int * 3)(-7, -7, -7)
    assert N.lib.rs_plan_tune(p.handle, None, 1, out, 3) == 0
    assert out[0] in (*range(7), 96, 98, 102, *range(256, 263)) and out[1] == -1 and out[2] == -1


@pytest.mark.parametrize("k,m,S,batch,off", [(10, 4, 100_003, 3, 3), (4, 2, 65_537, 5, 1),
                                             (12, 8, 16 * 496 + 9, 2, 6)])
def test_plan_tune_misaligned_split_layout(native_lib, k, m, S, batch, off):
    """On misaligned (Split-layout) shards rs_plan_tune chooses between the realigning
    kernel and the plain kernel in several tile orders; after tuning, encode and a decode
    with a Verify row stay bit-exact on every byte of every stripe."""
    import torch
    from callfs_amd.device import Plan
    n = k + m
    total = batch * n * S
    buf = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device="cuda:0")
    base = buf.data_ptr() + off
    ptrs = [base + (b * n + i) * S for b in range(batch) for i in range(n)]
    enc = Plan(k, m, S, batch, ptrs)
    names = enc.tune(reps=1)
    assert all(x in set(ALL_ORDER_NAMES) for x in names), names
    buf[off:off + total].copy_(torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda:0"))
    enc.launch()
    torch.cuda.synchronize()
    host = buf.cpu().numpy()[off:off + total].copy()
    for b in range(batch):
        st = host[b * n * S:(b + 1) * n * S]
        want = cref.encode([st[i * S:(i + 1) * S] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(st[(k + j) * S:(k + j + 1) * S], want[j]), (b, j)
    erase = [0, k - 1]  # m - 2 Verify rows
    dec = Plan(k, m, S, batch, ptrs, present=[i not in erase for i in range(n)])
    dec.tune(reps=1)
    for b in range(batch):
        for i in erase:
            s0 = off + (b * n + i) * S
            buf[s0:s0 + S].zero_()
    dec.launch()
    assert not dec.corrupt()
    assert np.array_equal(buf.cpu().numpy()[off:off + total], host)


@pytest.mark.parametrize("k,m,S,batch,erase", [
    (10, 4, 1 << 20, 3, None),          # bench shape, LDS kernel R = 4
    (10, 4, 100_003, 4, (5,)),          # one written + three compared rows, ragged tail
    (3, 2, 349_526, 3, None),           # v_perm launch (bounded by the LDS form)
    (10, 12, 65_536, 2, None),          # wide group R = 12
])
def test_plan_ceiling_modes_then_relaunch(native_lib, k, m, S, batch, erase):
    """rs_plan_launch_ceiling (bench.py's live roofline denominators): the read-only mode
    leaves every byte as it was; the write-only mode may overwrite the written rows, and
    relaunching the plan restores them bit-exactly; bad arguments are refused, and the
    A/B build's measurement modes (no-lookup, aligned-window probes) are RS_E_ARG
    in the product library."""
    import ctypes
    import torch
    from callfs_amd import _native as N
    from callfs_amd.device import Plan
    sb = _batch(k, m, S, batch, seed=S + 3 * k)
    enc = Plan.for_batch(sb)
    enc.launch()
    n = k + m
    present = None if erase is None else [i not in erase for i in range(n)]
    plan = enc if erase is None else Plan.for_batch(sb, present=present)
    before = sb.buf.clone()
    plan.launch_ceiling("read")
    torch.cuda.synchronize()
    assert torch.equal(sb.buf, before)
    for mode in ("nolookup", "write64", "write128", "write256", "read64", "read128", "read256"):
        assert N.lib.rs_plan_launch_ceiling(plan.handle, None, Plan.CEILINGS[mode]) == \
            N.RS_E_ARG, mode  # A/B-build modes (tools/callfs_rs_ab.h): not the product's
    torch.cuda.synchronize()
    assert torch.equal(sb.buf, before)
    for mode in ("write",):
        plan.launch_ceiling(mode)
        plan.corrupt()  # the no-lookup form compares junk: clear
        plan.launch()
        assert not plan.corrupt()
        torch.cuda.synchronize()
        assert torch.equal(sb.buf[:, :, :S], before[:, :, :S]), mode
    host = sb.buf[:, :, :S].cpu().numpy()
    want = cref.encode([host[0, i] for i in range(k)], k, m)
    for j in range(m):
        assert np.array_equal(host[0, k + j], want[j]), j
    assert N.lib.rs_plan_launch_ceiling(plan.handle, None, 9) == N.RS_E_ARG
    assert N.lib.rs_plan_launch_ceiling(plan.handle, None, -1) == N.RS_E_ARG
    assert N.lib.rs_plan_launch_ceiling(None, None, 0) == N.RS_E_ARG
    assert N.lib.rs_plan_groups(plan.handle) == max(1, -(-m // 16)) or erase is not None
    assert N.lib.rs_plan_groups(None) == 0


@pytest.mark.parametrize("k,m,S,batch,erase", [
    (10, 4, 1 << 20, 8, None),      # one LDS dispatch
    (20, 20, 65_536, 4, None),      # two launch groups: start on the first, stop on the last
    (4, 2, 10, 3, (0,)),            # S < 16: the byte kernel alone
])
def test_plan_launch_timed_events(native_lib, k, m, S, batch, erase):
    """rs_plan_launch_timed: the plan's first kernel dispatch records the start event and
    its last the stop event; the interval is positive and no longer than the same launch
    bracketed by stream events; outputs stay bit-exact. The ceiling modes time the same
    way. Events that do not exist yet are refused by the Python wrapper."""
    import torch
    from callfs_amd.device import Plan
    sb = _batch(k, m, S, batch, seed=S + 11 * k)
    present = None if erase is None else [i not in erase for i in range(k + m)]
    enc = Plan.for_batch(sb)
    plan = enc if erase is None else Plan.for_batch(sb, present=present)
    enc.launch()
    want = sb.buf.clone()
    stream = torch.cuda.current_stream()
    a, b, c, d = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    with pytest.raises(ValueError):
        plan.launch(stream, events=(a, b))
    for e in (a, b, c, d):
        e.record(stream)
    for _ in range(3):
        if erase is not None:
            sb.buf[:, list(erase)].zero_()
        c.record(stream)
        plan.launch(stream, events=(a, b))
        d.record(stream)
        torch.cuda.synchronize()
        kern, outer = a.elapsed_time(b), c.elapsed_time(d)
        assert 0 < kern <= outer * 1.02 + 0.005, (kern, outer)
    assert not plan.corrupt()
    assert torch.equal(sb.buf[:, :, :S], want[:, :, :S])
    if S >= 16:
        plan.launch_ceiling("read", stream, events=(a, b))
        torch.cuda.synchronize()
        assert a.elapsed_time(b) > 0


@pytest.mark.parametrize("k,m,S,batch", [(10, 4, 100_003, 3), (4, 2, 65_537, 5)])
def test_plan_ceiling_split_layout_stays_inside_written_shards(native_lib, k, m, S, batch):
    """On an upstream Split-layout batch (misaligned shards, pitch = S) the ceiling modes
    change nothing but the written shards: the write-only mode stores aligned blocks from
    each row's first 16-B boundary on, never a byte of a neighbouring input shard; the plan
    then restores its outputs bit-exactly."""
    import torch
    from callfs_amd.device import Plan, StripeBatch
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"), layout="split")
    sb.fill_random(S + k)
    enc = Plan.for_batch(sb)
    enc.launch()
    before = sb.buf.clone()
    for mode in ("read", "write"):
        enc.launch_ceiling(mode)
        torch.cuda.synchronize()
        assert torch.equal(sb.buf[:, :k], before[:, :k]), mode  # inputs untouched
        enc.launch()
        torch.cuda.synchronize()
        assert torch.equal(sb.buf, before), mode
    host = sb.buf.cpu().numpy()
    want = cref.encode([host[batch - 1, i] for i in range(k)], k, m)
    for j in range(m):
        assert np.array_equal(host[batch - 1, k + j], want[j]), j


@pytest.mark.parametrize("k,m,S,batch", [
    (10, 4, 100_003, 3),       # odd S: every data shard at its own offset, parity 64-B aligned
    (4, 2, 65_537, 5),
    (6, 3, 16 * 496 + 16 * 62 + 5, 4),  # realigning kernel's tile / wave edges
    (12, 4, 5_592_406 // 64, 2),        # even S
    (10, 4, 1 << 16, 3),                # 16 | S: every shard aligned
])
@pytest.mark.parametrize("how", ["rule", "tune", "realign-x32", "realign", "realign-tri-x32",
                                 "tri-x32", "tri-g2", "tri-x8", "tri-q8"])
def test_readall_layout_round_trip(native_lib, k, m, S, batch, how):
    """Upstream Split of an io.ReadAll body (StripeBatch layout "readall": data shards at
    pitch S inside the body, parity in 64-B AllocAligned buffers at a 64-B pitch): encode
    against the oracle on every stripe, then decodes of m data erasures, of erasures with
    Verify rows and of the parity alone restore every byte. how="tune": every plan first
    times each order its kernels offer; otherwise every plan is pinned to that kernel form
    (rs_plan_set_orders) where its launch offers it: the realigning kernel (ring or triple
    loads) or the triple loop's unaligned accesses."""
    import torch
    from callfs_amd import _native as N
    from callfs_amd.device import Plan, StripeBatch
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"), layout="readall")
    sb.fill_random(S + 3 * k)
    ptrs = sb.pointers()
    assert all(p % 64 == 0 for b in range(batch) for p in ptrs[b * (k + m) + k:(b + 1) * (k + m)])
    aligned = S % 16 == 0  # every data shard 16-B aligned: no realigning form

    def ready(plan, outputs_aligned=True):
        if how == "tune":
            plan.tune(reps=1)
        elif how != "rule":
            try:
                plan.set_orders([how] * int(N.lib.rs_plan_groups(plan.handle)))
            except N.NativeError as e:  # not offered for this launch: the rule's kernel
                assert e.code == N.RS_E_ARG
                assert aligned or not how.startswith("realign"), how  # misaligned: offered
        return plan

    ready(Plan.for_batch(sb)).launch()
    torch.cuda.synchronize()
    host = sb.gather().cpu().numpy()
    for b in range(batch):
        want = cref.encode([host[b, i] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(host[b, k + j], want[j]), (b, j)
    for erase in (list(range(0, k, max(1, k // m)))[:m], [1, k], list(range(k, k + m))):
        for i in erase:
            sb.zero_shard(i)
        dec = ready(Plan.for_batch(sb, present=[i not in erase for i in range(k + m)]),
                    outputs_aligned=min(erase) >= k)
        dec.launch()
        assert not dec.corrupt(), erase
        assert np.array_equal(sb.gather().cpu().numpy(), host), erase


@pytest.mark.parametrize("k,m,S,batch", [
    (10, 4, 100_003, 3),
    (10, 4, 1_677_722 + 1, 2),          # 205 tiles per shard: the readall rule's Q8 band
    (6, 3, 16 * 496 + 16 * 62 + 5, 4),
    (12, 4, 5_592_406 // 64, 2),
])
@pytest.mark.parametrize("how", ["rule", "tune", "tri-x32", "tri-q8", "tri-g2", "realign-x32", "bs-x32", "bs-g8"])
def test_readall_decode_into_fresh_buffers(native_lib, k, m, S, batch, how):
    """The decode CallFS runs on an io.ReadAll body (bench.py --layout readall --decode-into
    fresh): survivors at odd offsets in the body, the erased shards rebuilt into buffers of
    their own (64-B pitch, 256-B aligned), as upstream Reconstruct allocates missing shards.
    Misaligned inputs with aligned outputs take the unaligned triples (tri_unaligned_order);
    every rebuilt shard equals the encoded original, for each pinned form the launch offers."""
    import torch
    from callfs_amd import _native as N
    from callfs_amd.device import Plan, StripeBatch, _aligned_empty
    n = k + m
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"), layout="readall")
    sb.fill_random(S + 7 * k)
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    host = sb.gather().cpu().numpy()
    for b in range(batch):
        want = cref.encode([host[b, i] for i in range(k)], k, m)
        assert all(np.array_equal(host[b, k + j], want[j]) for j in range(m)), b
    fp = -(-S // 64) * 64
    for erase in (list(range(0, k, max(1, k // m)))[:m], [1, k], [0, 3]):
        fresh = _aligned_empty((batch, len(erase), fp), 256, torch.device("cuda:0"))
        fresh.fill_(0xA5)
        ptrs = list(sb.pointers())
        for b in range(batch):
            for j, i in enumerate(erase):
                ptrs[b * n + i] = fresh[b, j].data_ptr()
        dec = Plan(k, m, S, batch, ptrs, present=[i not in erase for i in range(n)])
        if how == "tune":
            dec.tune(reps=1)
        elif how != "rule":
            try:
                dec.set_orders([how] * int(N.lib.rs_plan_groups(dec.handle)))
            except N.NativeError as e:  # not offered for this launch: the rule's kernel
                assert e.code == N.RS_E_ARG
        dec.launch()
        assert not dec.corrupt(), erase
        got = fresh.cpu().numpy()
        for b in range(batch):
            for j, i in enumerate(erase):
                assert np.array_equal(got[b, j, :S], host[b, i]), (erase, b, i)
        del dec, fresh


@pytest.mark.parametrize("k,m,L", [(10, 4, 10 * 1000 + 7), (4, 2, 4 * 37 + 1), (16, 4, 4096)])
def test_small_path_verify_masks_the_tail_vector(codec, k, m, L):
    """Small calls take the one-dispatch path, whose last 16-B vector per shard runs past S
    (padding in staging): a flipped last byte of a compared parity shard must be reported,
    while the padding is never compared (clean decodes of odd-S objects stay clean)."""
    from callfs_amd import ErasureProfile, ErrShardCorrupted
    p = ErasureProfile(k, m)
    data = rnd(L + k, L)
    full = [bytes(s) for s in codec.encode(data, p)]
    S = len(full[0])
    sh = [None if i == 0 else full[i] for i in range(k + m)]
    assert codec.decode(sh, p, L) == data  # k-1 data + m parity: m-1 compared rows, clean
    for pos in (S - 1, 0):
        bad = [bytearray(x) for x in full]
        bad[k + m - 1][pos] ^= 0x80
        sh = [None if i == 0 else bad[i] for i in range(k + m)]
        with pytest.raises(ErrShardCorrupted):
            codec.decode(sh, p, L)


@pytest.mark.parametrize("k,m,S,B", [(10, 4, 960, 150),    # 150 blocks in y, one in x
                                     (10, 4, 16000, 9),    # 4 x 9 blocks
                                     (4, 2, 340_000, 1),   # 84 blocks, one stripe
                                     (16, 4, 6000, 16)])   # 2 x 16 blocks, 2 loads rounds
def test_small_path_every_byte_right_after_flag(native_lib, k, m, S, B):
    """One-dispatch calls of close to the 2 MiB staging limit spread over many blocks: the
    host reads outputs as soon as the kernel's completion flag is released, so every
    block's (every wave's) PCIe stores must be visible by then. Repeated back to back,
    every byte of every stripe checked against the oracle."""
    from callfs_amd import erasure as E
    assert ((S + 15) // 16 * 16) * (k + m) * B <= 2 << 20  # one dispatch
    rng = np.random.default_rng(S * B + k)
    for rep in range(6):
        stripes = [[rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] for _ in range(B)]
        parity, status = E.encode_batch(stripes, k, m)
        assert status == [0] * B
        for b in range(B):
            want = cref.encode(stripes[b], k, m)
            for j in range(m):
                assert bytes(parity[b][j]) == bytes(want[j]), (rep, b, j)


@pytest.mark.parametrize("k,m,S", [
    (10, 4, 16 * 512 * 3 + 5),          # last tile full: the tail in tile 0's wave 0
    (10, 4, 16 * (512 * 3 + 100) + 7),  # last tile partial: its idle last wave takes the tail
    (10, 4, 16 * (512 * 2 + 448) + 9),  # 448 vectors: the last wave exactly idle
    (10, 4, 16 * (512 * 2 + 449) + 3),  # 449: the last wave holds one vector -> tile 0
    (10, 4, 16 * 40 + 11),              # one partial tile: first and last tile coincide
    (10, 4, 16 * (512 * 40 + 100) + 7),  # 41 tiles per stripe (> 32): tile 0's wave 0
    (6, 3, 16 * (512 * 31 + 60) + 1),    # 32 tiles, partial last: the idle last wave
    (3, 2, 16 * (512 + 77) + 13),       # v_perm kernel (k <= 3), partial last tile
    (3, 2, 16 * 1024 + 1),              # v_perm kernel, full last tile
    (12, 8, 16 * (512 * 4 + 300) + 15),  # R = 8, triple loads at this size
    (20, 16, 16 * (512 + 10) + 2),       # wide group (16-byte entries)
])
def test_ragged_tail_wave_placement(native_lib, k, m, S):
    """The S % 16 tail bytes of every stripe go to the idle last wave of the stripe's last
    tile when that tile is partial and a stripe has at most 32 tiles, else to wave 0 of its
    first tile (rs_apply.hpp tail_lane, rs_kernels.hip tail_mode): encode every byte against the oracle, and a decode with Verify rows flags
    a flipped last byte (which only the tail wave computes) in exactly its stripe."""
    import torch
    from callfs_amd.device import Plan
    batch = 3
    sb = _batch(k, m, S, batch, seed=S)
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    h = sb.buf[:, :, :S].cpu().numpy()
    for b in range(batch):
        want = cref.encode([h[b, i] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(h[b, k + j], want[j]), (b, j)
    n = k + m
    present = [i != 0 for i in range(n)]  # one erasure: m - 1 Verify rows
    dec = Plan.for_batch(sb, present=present)
    sb.buf[:, 0].zero_()
    dec.launch()
    assert not dec.corrupt()
    assert np.array_equal(sb.buf[:, :, :S].cpu().numpy(), h)
    sb.buf[1, n - 1, S - 1] ^= 0x20
    dec.launch()
    assert dec.corrupt_stripes() == [1]


@pytest.mark.parametrize("k", [6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 32, 65])
@pytest.mark.parametrize("m", [1, 2, 4])
def test_plan_double_buffered_triples_vs_oracle(native_lib, k, m):
    """R <= 4 launches with K >= 6 run the triple loop double-buffered in two register sets
    (Policy::WIX 3): its straight-line tails cover one or two remaining triples and K % 3 =
    0, 1, 2 leftover shards. Every form, in three orders with triple instances, against the
    oracle on every byte of every stripe, with a ragged tail."""
    import torch
    from callfs_amd.device import Plan
    S, batch, n = 65_536 + 16 * 37 + 5, 3, k + m
    pitch = (S + 255) // 256 * 256
    buf = torch.randint(0, 256, (batch, n, pitch), dtype=torch.uint8, device="cuda:0")
    ptrs = [buf[b, i].data_ptr() for b in range(batch) for i in range(n)]
    h = buf.cpu().numpy()
    want = [cref.encode([h[b, i, :S] for i in range(k)], k, m) for b in range(batch)]
    for order in ("tri", "tri-g2", "tri-x8"):
        buf[:, k:].zero_()
        plan = Plan(k, m, S, batch, ptrs)
        plan.set_orders([order])
        plan.launch()
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        for b in range(batch):
            for j in range(m):
                assert np.array_equal(got[b, k + j, :S], want[b][j]), (order, b, j)


@pytest.mark.parametrize("k,m,S,batch", [
    (8, 4, 2 << 20, 3),            # K 7..9, 1-2 MiB: double-buffered triples in G2
    (8, 4, (8 << 20) - 16 * 3 - 1, 2),  # K 7..9 above 2 MiB: the ring, consecutive (ragged tail)
    (10, 4, (2 << 20) + 7, 3),     # K >= 10 above 1 MiB: the ring
    (8, 8, 2 << 20, 3),            # R 5..8, 1-2 MiB, K < 10: triples, consecutive
    (10, 8, 1_677_722, 3),         # R 5..8, K 10..12 to 2 MiB: triples in Q8
    (10, 8, 6_710_887 // 2, 2),    # R 5..8 to 8 MiB: triples in X32
    (8, 8, 131_072, 5),            # R 5..8 up to 256 KiB: triples in G2
    (20, 4, 52_429, 9),            # R <= 4, K > 16, small: double-buffered triples in G2
    (20, 4, 838_861, 3),           # K > 16, 256 KiB - 1 MiB: the ring, consecutive
    (32, 8, 2 << 20, 2),           # K > 16 with 8 rows above 1 MiB: the ring, consecutive
])
def test_planar_rule_forms_vs_oracle(native_lib, k, m, S, batch):
    """The round-5 rule (tile_order.hpp, fitted on the planar layout) picks a different form
    or order on these shapes than round 4's: the rule's own launch, on a planar batch,
    against the oracle on every byte of every stripe, and the m-erasure decode of the data
    shards in front restores them."""
    import torch
    from callfs_amd.device import Plan, StripeBatch
    sb = StripeBatch(k, m, S, batch, torch.device("cuda:0"), layout="planar")
    sb.fill_random(S + 7 * k + m)
    Plan.for_batch(sb).launch()
    torch.cuda.synchronize()
    h = sb.gather().cpu().numpy()
    for b in range(batch):
        want = cref.encode([h[b, i] for i in range(k)], k, m)
        for j in range(m):
            assert np.array_equal(h[b, k + j], want[j]), (b, j)
    erase = list(range(min(m, k)))
    for i in erase:
        sb.zero_shard(i)
    dec = Plan.for_batch(sb, present=[i not in erase for i in range(k + m)])
    dec.launch()
    assert not dec.corrupt()
    assert np.array_equal(sb.gather().cpu().numpy(), h)
