"""The oracle itself: pinned by the upstream known-answer values and the
reference's codec_test.go scenarios, and the two restatements (numpy, C) agree."""
import numpy as np
import pytest

from oracle import cref
from oracle import rs_oracle as o


def test_kats():
    o.check_kats()


def test_gal_mul_kat():
    for (a, b), want in o.KATS["gal_mul"]:
        assert o.gal_mul(a, b) == want
        assert cref.lib().orc_gal_mul(a, b) == want


def test_gal_exp_kat():
    for (a, n), want in o.KATS["gal_exp"]:
        assert o.gal_exp(a, n) == want


def test_one_encode_kat():
    k, m, data, want = o.KATS["one_encode"]
    par = cref.encode([np.array(d, np.uint8) for d in data], k, m)
    assert [list(map(int, p)) for p in par] == want


@pytest.mark.parametrize("km", list(o.KATS["parity_rows"]))
def test_parity_rows_kat(km):
    k, m = km
    assert o.parity_matrix(k, m) == o.KATS["parity_rows"][km]
    assert cref.encode_matrix(k, m)[k:].tolist() == o.KATS["parity_rows"][km]


@pytest.mark.parametrize("k,m", [(1, 1), (2, 1), (3, 2), (4, 2), (10, 4), (16, 4), (5, 5),
                                 (17, 3), (64, 16), (200, 56)])
def test_matrix_restatements_agree(k, m):
    E = o.encode_matrix(k, m)
    assert cref.encode_matrix(k, m).tolist() == E
    assert E[:k] == [[1 if i == j else 0 for j in range(k)] for i in range(k)]


def test_small_data_hi():
    # codec_test.go:123-142 TestEncodeSmallData + SURVEY 8c: "hi", RS(4,2)
    sh = o.codec_encode(b"hi", 4, 2)
    assert [bytes(s) for s in sh] == [b"h", b"i", b"\0", b"\0", b"\x19", b"\x1e"]
    assert o.codec_decode(list(sh), 4, 2, 2) == b"hi"


def test_codec_test_scenarios():
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, 100 * 1024, dtype=np.uint8).tobytes()
    sh = o.codec_encode(data, 4, 2)
    assert len(sh) == 6
    assert o.codec_decode(list(sh), 4, 2, len(data)) == data
    deg = list(sh)
    deg[1] = None
    deg[4] = None
    assert o.codec_decode(deg, 4, 2, len(data)) == data
    bad = list(sh)
    bad[0] = bad[2] = bad[4] = None
    with pytest.raises(o.ErrTooFewShards):
        o.codec_decode(bad, 4, 2, len(data))
    with pytest.raises(o.ErrInvalidProfile):
        o.codec_encode(b"test", 0, 2)
    with pytest.raises(o.ErrInvalidProfile):
        o.codec_encode(b"test", 4, 0)
    with pytest.raises(o.ErrShortData):
        o.codec_encode(b"", 4, 2)


def test_verify_detects_flipped_parity_bit():
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 4096, dtype=np.uint8).tobytes()
    sh = o.codec_encode(data, 10, 4)
    sh[12] = sh[12].copy()
    sh[12][100] ^= 1
    assert not o.verify(sh, 10, 4)
    with pytest.raises(o.ErrShardCorrupted):
        o.codec_decode(list(sh), 10, 4, len(data))


@pytest.mark.parametrize("erase", [(0, 1, 2, 3), (0, 3, 7, 12), (10, 11, 12, 13), (5,), ()])
def test_rs10_4_erasures_c_vs_numpy(erase):
    rng = np.random.default_rng(11)
    k, m, S = 10, 4, 5003
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    par = cref.encode(data, k, m)
    par_np = o.apply_rows(o.parity_matrix(k, m), data)
    assert all((a == b).all() for a, b in zip(par, par_np))
    full = data + par
    present = [i not in erase for i in range(k + m)]
    shards = [s if present[i] else None for i, s in enumerate(full)]
    rec_c = cref.reconstruct(list(shards), present, k, m)
    rec_np = o.reconstruct([None if s is None else s.copy() for s in shards], k, m)
    for a, b, c in zip(rec_c, rec_np, full):
        assert (a == c).all() and (np.asarray(b) == c).all()


def test_simd_baseline_matches_scalar():
    rng = np.random.default_rng(5)
    for k, m, S in [(10, 4, 1 << 16), (3, 2, 349526), (16, 4, 4096 + 17), (4, 9, 1000)]:
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        a = cref.encode(data, k, m)
        b = cref.encode(data, k, m, simd=True, nthreads=4)
        assert all((x == y).all() for x, y in zip(a, b)), (k, m, S)


def test_decode_rows_oracle_consistency():
    k, m = 10, 4
    present = [True] * 14
    for e in (0, 3, 7, 12):
        present[e] = False
    valid, missing, rows = o.decode_rows(k, m, present)
    assert valid == [1, 2, 4, 5, 6, 8, 9, 10, 11, 13]
    assert missing == [0, 3, 7, 12]
    rng = np.random.default_rng(0)
    data = [rng.integers(0, 256, 257, dtype=np.uint8) for _ in range(k)]
    full = data + o.apply_rows(o.parity_matrix(k, m), data)
    got = o.apply_rows(rows, [full[i] for i in valid])
    for idx, g in zip(missing, got):
        assert (g == full[idx]).all()


def test_golden_vectors_reproduce_with_c_oracle():
    """tests/golden/vectors.json (made by the numpy oracle) re-derived by the
    independent C restatement."""
    import hashlib
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vectors.json")
    vec = json.load(open(path))
    for case in vec["raw"]:
        k, m = case["k"], case["m"]
        data = bytes.fromhex(case["data"])
        S = (len(data) + k - 1) // k
        buf = np.zeros(S * k, np.uint8)
        buf[: len(data)] = np.frombuffer(data, np.uint8)
        dsh = [buf[i * S:(i + 1) * S] for i in range(k)]
        got = [d.tobytes().hex() for d in dsh] + [p.tobytes().hex() for p in cref.encode(dsh, k, m)]
        assert got == case["shards"], case["name"]
    for case in vec["digest"]:
        if case["len"] > (16 << 20):
            continue  # the 64 MiB case is exercised on the GPU box
        k, m = case["k"], case["m"]
        data = np.random.default_rng(case["seed"]).integers(0, 256, case["len"], dtype=np.uint8)
        S = (len(data) + k - 1) // k
        buf = np.zeros(S * k, np.uint8)
        buf[: len(data)] = data
        dsh = [buf[i * S:(i + 1) * S] for i in range(k)]
        sh = dsh + cref.encode(dsh, k, m, simd=True, nthreads=4)
        assert [hashlib.sha256(s.tobytes()).hexdigest() for s in sh] == case["shard_sha256"]


def test_configs0_rs3_2_1mib_encode_verify():
    """BASELINE.json configs[0]: RS(3,2) encode + verify of a 1 MiB object on the CPU
    (erasure/codec_test.go's round trip at that size): S = 349,526 with 2 bytes of Split
    padding, Verify passes, Decode with every shard present returns the object, and the
    per-shard SHA-256 equal the golden fixture of the same seeded input."""
    import hashlib
    import json
    import os
    vec = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "vectors.json")))
    case = next(c for c in vec["digest"] if c["name"] == "1mib_rs3_2")
    data = np.random.default_rng(case["seed"]).integers(0, 256, case["len"], dtype=np.uint8).tobytes()
    shards = o.codec_encode(data, 3, 2)
    assert [len(s) for s in shards] == [349_526] * 5
    assert bytes(np.asarray(shards[2])[-2:]) == b"\0\0"
    assert o.verify(shards, 3, 2)
    assert [hashlib.sha256(np.asarray(s).tobytes()).hexdigest() for s in shards] == case["shard_sha256"]
    assert o.codec_decode(list(shards), 3, 2, len(data)) == data


# ---- checks that need no recalled value --------------------------

def _clmul_mod_11d(a, b):
    """Carry-less product of byte arrays reduced mod x^8+x^4+x^3+x^2+1 (0x11D): the
    field's definition, with no log/exp tables."""
    a = a.astype(np.int64)
    b = b.astype(np.int64)
    acc = np.zeros(np.broadcast(a, b).shape, np.int64)
    for i in range(8):
        acc ^= np.where((b >> i) & 1, a << i, 0)
    for bit in range(14, 7, -1):
        acc ^= np.where((acc >> bit) & 1, 0x11D << (bit - 8), 0)
    return acc


def _independent_log_exp():
    """log/exp of the generator 2 built by repeated clmul (not the oracle's tables)."""
    exp = np.zeros(255, np.int64)
    log = np.full(256, -1, np.int64)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x = int(_clmul_mod_11d(np.array(x), np.array(2)))
    assert sorted(exp.tolist()) == list(range(1, 256))  # 2 generates GF(2^8)*
    return exp, log


def test_gal_mul_exhaustive_vs_clmul():
    a, b = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    want = _clmul_mod_11d(a, b)
    got_np = np.array([[o.gal_mul(x, y) for y in range(256)] for x in range(256)])
    assert (got_np == want).all()
    L = cref.lib()
    got_c = np.array([[L.orc_gal_mul(x, y) for y in range(256)] for x in range(256)])
    assert (got_c == want).all()


def _lagrange_matrix(k, exp, log):
    """E[r][i] = prod_{j<k, j!=i} (r ^ j) / (i ^ j) for r in 0..255 (r < k: identity
    rows): the unique matrix mapping values at the points 0..k-1 of a polynomial of
    degree < k to its value at r, which is what E = V . inv(V[0:k]) is, V[r][c] = r^c."""
    E = np.zeros((256, k), np.int64)
    E[np.arange(k), np.arange(k)] = 1
    if k == 256:
        return E
    i = np.arange(k)
    r = np.arange(k, 256)
    lr = log[r[:, None] ^ i[None, :]]            # (256-k, k): log(r ^ j), all nonzero
    tot = lr.sum(axis=1)                           # sum over every j < k
    li = log[np.where(i[:, None] == i[None, :], 1, i[:, None] ^ i[None, :])]
    li[i, i] = 0                                   # skip j == i
    den = li.sum(axis=1)
    E[k:] = exp[(tot[:, None] - lr - den[None, :]) % 255]
    return E


def test_encode_matrix_lagrange_closed_form_every_k():
    """E's rows do not depend on m, so E(k, 256-k) covers every (k, m) with k+m <= 256.
    Checked for every k against the C oracle, and for k <= 24 against the numpy oracle
    (pure-Python Gauss-Jordan)."""
    exp, log = _independent_log_exp()
    for k in range(1, 256):
        want = _lagrange_matrix(k, exp, log)
        assert (cref.encode_matrix(k, 256 - k).astype(np.int64) == want).all(), k
        if k <= 24:
            assert (np.array(o.encode_matrix(k, 256 - k)) == want).all(), k


def test_product_encode_matrix_lagrange_every_k(native_lib):
    """The product's host matrix code (gf256.hpp via rs_encode_matrix, no device)."""
    from callfs_amd.erasure import encode_matrix
    exp, log = _independent_log_exp()
    for k in range(1, 256):
        assert (encode_matrix(k, 256 - k).astype(np.int64) == _lagrange_matrix(k, exp, log)).all(), k
