"""CPU oracle for the CallFS Reed-Solomon erasure-coding path.

TEST INFRASTRUCTURE ONLY. Nothing in ``callfs_amd/`` may import, call or link this
module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker.

What it restates
----------------
``erasure/codec.go`` (``Codec.Encode`` 21-41, ``Codec.Decode`` 45-78) drives
``github.com/klauspost/reedsolomon v1.13.3`` (``go.mod:13``; pinned by
``go.sum:157-158``). That module is not present in ``/root/reference`` and there is
no Go toolchain or network here, so the library's published algorithm is restated
from scratch:

* GF(2^8), polynomial 0x11D, generator 2: ``galMultiply``/``galDivide``/``galExp``
  (upstream ``galois.go``).
* ``buildMatrix``: ``E = V . inv(V[0:k])`` with ``V[r][c] = galExp(r, c)``
  (upstream ``reedsolomon.go`` buildMatrix / ``matrix.go`` vandermonde, invert).
* ``Split`` zero padding with ``S = ceil(L/k)`` (upstream ``Split``; called at
  ``erasure/codec.go:31``).
* ``Encode``: ``parity_j = XOR_i P[j][i] * data_i`` (``codec.go:36``).
* ``Reconstruct``: first k present shards in index order, ``inv(E[valid])`` for data,
  parity re-encoded from the reconstructed data (``codec.go:55``).
* ``Verify``: full parity recompute + compare (``codec.go:59``).
* ``Decode`` join/trim and error precedence (``codec.go:45-78``).

Parity pinning
--------------
The reference's own tests (``erasure/codec_test.go:9-142``) pin only round trips
and error identity, never parity bytes. The oracle is therefore pinned by the
upstream known-answer values recorded in SURVEY.md section 8(c) (``galMultiply``,
``galExp``, ``galMulSlice``, ``TestOneEncode`` RS(5,5), and the RS(3,2), RS(4,2),
RS(10,4) parity rows); see ``KATS`` below and ``tests/test_oracle.py``.
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D
GEN = 2

# --------------------------------------------------------------------------------------
# GF(2^8) field (upstream galois.go: logTable/expTable generated from 0x11D, alpha=2)
# --------------------------------------------------------------------------------------


def _build_tables():
    exp = np.zeros(510, dtype=np.int32)
    log = np.zeros(256, dtype=np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    exp[255:510] = exp[0:255]
    return exp, log


EXP, LOG = _build_tables()


def gal_mul(a: int, b: int) -> int:
    """upstream galMultiply: 0 if either operand is 0, else exp[log a + log b]."""
    if a == 0 or b == 0:
        return 0
    return int(EXP[LOG[a] + LOG[b]])


def gal_div(a: int, b: int) -> int:
    """upstream galDivide (b != 0)."""
    if a == 0:
        return 0
    if b == 0:
        raise ZeroDivisionError("gal_div by zero")
    return int(EXP[(LOG[a] - LOG[b]) % 255])


def gal_exp(a: int, n: int) -> int:
    """upstream galExp: n==0 -> 1 (also for a==0); a==0 -> 0."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(int(LOG[a]) * n) % 255])


def _build_mul_table():
    t = np.zeros((256, 256), dtype=np.uint8)
    for a in range(1, 256):
        la = LOG[a]
        t[a, 1:] = EXP[(la + LOG[1:]) % 255]
    return t


MUL = _build_mul_table()


def gal_mul_slice(c: int, data: np.ndarray) -> np.ndarray:
    """upstream galMulSlice: out[i] = c * in[i]."""
    return MUL[c][np.asarray(data, dtype=np.uint8)]


# --------------------------------------------------------------------------------------
# Matrices (upstream matrix.go)
# --------------------------------------------------------------------------------------


def mat_mul(a, b):
    n, kk = len(a), len(a[0])
    assert kk == len(b)
    p = len(b[0])
    out = [[0] * p for _ in range(n)]
    for r in range(n):
        for c in range(p):
            v = 0
            for i in range(kk):
                v ^= gal_mul(a[r][i], b[i][c])
            out[r][c] = v
    return out


class SingularMatrix(Exception):
    pass


def mat_inv(m):
    """Gauss-Jordan inversion over GF(2^8) (upstream matrix.Invert / gaussianElimination)."""
    n = len(m)
    work = [list(row) + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(m)]
    for r in range(n):
        if work[r][r] == 0:
            for below in range(r + 1, n):
                if work[below][r] != 0:
                    work[r], work[below] = work[below], work[r]
                    break
        if work[r][r] == 0:
            raise SingularMatrix("matrix is singular")
        if work[r][r] != 1:
            scale = gal_div(1, work[r][r])
            work[r] = [gal_mul(scale, v) for v in work[r]]
        for other in range(n):
            if other != r and work[other][r] != 0:
                f = work[other][r]
                work[other] = [v ^ gal_mul(f, w) for v, w in zip(work[other], work[r])]
    return [row[n:] for row in work]


def vandermonde(rows: int, cols: int):
    return [[gal_exp(r, c) for c in range(cols)] for r in range(rows)]


def encode_matrix(k: int, m: int):
    """upstream buildMatrix: E = V . inv(V[0:k]); rows 0..k-1 are the identity."""
    v = vandermonde(k + m, k)
    top_inv = mat_inv(v[:k])
    return mat_mul(v, top_inv)


def parity_matrix(k: int, m: int):
    return encode_matrix(k, m)[k:]


# --------------------------------------------------------------------------------------
# Errors (erasure/errors.go:7-10 + upstream reedsolomon error values)
# --------------------------------------------------------------------------------------


class OracleError(Exception):
    code = "error"


def _err(name, msg):
    return type(name, (OracleError,), {"code": name, "msg": msg})


ErrInvalidProfile = _err("ErrInvalidProfile", "erasure: invalid erasure profile parameters (code 3054)")
ErrInsufficientShards = _err("ErrInsufficientShards", "erasure: insufficient shards for reconstruction (code 3050)")
ErrShardCorrupted = _err("ErrShardCorrupted", "erasure: shard checksum mismatch (code 3051)")
ErrShortData = _err("ErrShortData", "not enough data to fill the number of requested shards")
ErrTooFewShards = _err("ErrTooFewShards", "too few shards given")
ErrShardNoData = _err("ErrShardNoData", "no shard data")
ErrShardSize = _err("ErrShardSize", "shard sizes do not match")
ErrUnsupported = _err("ErrUnsupported", "k+m > 256 uses the Leopard GF(2^16) codec")


# --------------------------------------------------------------------------------------
# Codec path (erasure/codec.go)
# --------------------------------------------------------------------------------------


def shard_size(length: int, k: int) -> int:
    return (length + k - 1) // k


def split(data: bytes, k: int, m: int):
    """upstream Split: S = ceil(L/k); data zero-padded to k*S; parity buffers zeroed."""
    if len(data) == 0:
        raise ErrShortData()
    s = shard_size(len(data), k)
    buf = np.zeros((k + m) * s, dtype=np.uint8)
    buf[: len(data)] = np.frombuffer(bytes(data), dtype=np.uint8)
    return [buf[i * s:(i + 1) * s].copy() for i in range(k + m)]


def apply_rows(rows, inputs):
    """out_r[b] = XOR_i rows[r][i] * inputs[i][b]."""
    outs = []
    for row in rows:
        acc = np.zeros_like(inputs[0])
        for c, x in zip(row, inputs):
            if c == 0:
                continue
            acc ^= MUL[c][x]
        outs.append(acc)
    return outs


def encode_shards(shards, k: int, m: int):
    """upstream Encode: fill parity shards k..k+m-1 in place."""
    p = parity_matrix(k, m)
    par = apply_rows(p, shards[:k])
    for j in range(m):
        shards[k + j] = par[j]
    return shards


def codec_encode(data: bytes, k: int, m: int):
    """erasure/codec.go:21-41 Codec.Encode."""
    if k < 1 or m < 1:
        raise ErrInvalidProfile()
    if k + m > 256:
        raise ErrUnsupported()
    shards = split(data, k, m)
    return encode_shards(shards, k, m)


def _check_shards(shards, nilok: bool):
    size = 0
    for s in shards:
        if s is not None and len(s) != 0:
            size = len(s)
            break
    if size == 0:
        raise ErrShardNoData()
    for s in shards:
        ln = 0 if s is None else len(s)
        if ln != size and (ln != 0 or not nilok):
            raise ErrShardSize()
    return size


def reconstruct(shards, k: int, m: int):
    """upstream Reconstruct (dataOnly=false), first-k-present rule. Mutates shards."""
    n = k + m
    if len(shards) != n:
        raise ErrTooFewShards()
    size = _check_shards(shards, True)
    present = [s is not None and len(s) != 0 for s in shards]
    if all(present):
        return shards
    if sum(present) < k:
        raise ErrTooFewShards()
    valid = [i for i in range(n) if present[i]][:k]
    e = encode_matrix(k, m)
    dec = mat_inv([e[i] for i in valid])
    sub = [np.asarray(shards[i], dtype=np.uint8) for i in valid]
    for i in range(k):
        if not present[i]:
            shards[i] = apply_rows([dec[i]], sub)[0]
    p = e[k:]
    data = [np.asarray(shards[i], dtype=np.uint8) for i in range(k)]
    for j in range(m):
        if not present[k + j]:
            shards[k + j] = apply_rows([p[j]], data)[0]
    assert all(len(s) == size for s in shards)
    return shards


def verify(shards, k: int, m: int) -> bool:
    """upstream Verify: recompute parity from data shards and compare."""
    if len(shards) != k + m:
        raise ErrTooFewShards()
    _check_shards(shards, False)
    p = parity_matrix(k, m)
    data = [np.asarray(s, dtype=np.uint8) for s in shards[:k]]
    par = apply_rows(p, data)
    return all(np.array_equal(par[j], np.asarray(shards[k + j], dtype=np.uint8)) for j in range(m))


def codec_decode(shards, k: int, m: int, original_size: int) -> bytes:
    """erasure/codec.go:45-78 Codec.Decode (mutates shards like the Go code)."""
    if k < 1 or m < 1:
        raise ErrInvalidProfile()
    if k + m > 256:
        raise ErrUnsupported()
    reconstruct(shards, k, m)
    if not verify(shards, k, m):
        raise ErrShardCorrupted()
    buf = b"".join(np.asarray(shards[i], dtype=np.uint8).tobytes() for i in range(k))
    if len(buf) < original_size:
        raise ErrInsufficientShards()
    return buf[:original_size]


def decode_rows(k: int, m: int, present):
    """Composite matrix the fused GPU decode applies: rows over the first k present
    shards that yield every missing shard (data rows of inv(E[valid]); parity rows
    P[j] . inv(E[valid])). Returns (valid, missing, rows). Used by tests to check the
    library's host-side matrix builder."""
    n = k + m
    valid = [i for i in range(n) if present[i]][:k]
    e = encode_matrix(k, m)
    dec = mat_inv([e[i] for i in valid])
    missing = [i for i in range(n) if not present[i]]
    rows = []
    for i in missing:
        rows.append(dec[i] if i < k else mat_mul([e[i]], dec)[0])
    return valid, missing, rows


# --------------------------------------------------------------------------------------
# Known-answer values (upstream reedsolomon tests)
# --------------------------------------------------------------------------------------

# Provenance (none of these files is in /root/reference; the values are upstream's
# published test constants for klauspost/reedsolomon v1.13.3, recalled, as SURVEY.md
# 8(c) records -- nothing reference-held pins parity bytes):
#   gal_mul, gal_exp, gal_mul_slice  galois_test.go TestGalois (galMultiply, galExp,
#                                    galMulSlice with c = 25)
#   one_encode                       reedsolomon_test.go TestOneEncode, RS(5,5)
#   parity_rows                      rows of buildMatrix's E[k:] for these profiles
# tests/test_oracle.py also checks the field and the matrix construction without any
# recalled value: every product against a carry-less multiply reduced mod 0x11D, and
# every row of E = V . inv(V[0:k]) for every k against the Lagrange closed form.
KATS = {
    "gal_mul": [((3, 4), 12), ((7, 7), 21), ((23, 45), 41)],
    "gal_exp": [((2, 2), 4), ((5, 20), 235), ((13, 7), 43)],
    "gal_mul_slice": (
        25,
        [0, 1, 2, 3, 4, 5, 6, 10, 50, 100, 150, 174, 201, 255, 99, 32, 67, 85, 200],
        [0x00, 0x19, 0x32, 0x2B, 0x64, 0x7D, 0x56, 0xFA, 0xB8, 0x6D, 0xC7, 0x85, 0xC3,
         0x1F, 0x22, 0x07, 0x25, 0xFE, 0xDA],
    ),
    # upstream TestOneEncode: RS(5,5)
    "one_encode": (
        5, 5,
        [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
        [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]],
    ),
    "parity_rows": {
        (3, 2): [[1, 1, 1], [15, 8, 6]],
        (4, 2): [[27, 28, 18, 20], [28, 27, 20, 18]],
        (10, 4): [
            [129, 150, 175, 184, 210, 196, 254, 232, 3, 2],
            [150, 129, 184, 175, 196, 210, 232, 254, 2, 3],
            [191, 214, 98, 10, 6, 111, 223, 183, 5, 4],
            [214, 191, 10, 98, 111, 6, 183, 223, 4, 5],
        ],
    },
}


def check_kats() -> None:
    """Raise AssertionError unless every known-answer value reproduces."""
    for (a, b), want in KATS["gal_mul"]:
        assert gal_mul(a, b) == want, ("gal_mul", a, b)
    for (a, n), want in KATS["gal_exp"]:
        assert gal_exp(a, n) == want, ("gal_exp", a, n)
    c, inp, want = KATS["gal_mul_slice"]
    assert list(gal_mul_slice(c, inp)) == want
    k, m, data, want = KATS["one_encode"]
    shards = [np.array(d, dtype=np.uint8) for d in data] + [np.zeros(2, np.uint8)] * m
    encode_shards(shards, k, m)
    assert [list(map(int, s)) for s in shards[k:]] == want
    for (k, m), rows in KATS["parity_rows"].items():
        assert parity_matrix(k, m) == rows, ("parity_rows", k, m)
