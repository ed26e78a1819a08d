"""Host-side mirror of CallFS's Go `erasure` codec, backed by the HIP C ABI.

Same names, argument meaning and error behaviour as the reference:

    Go (erasure/)                                   here
    ErasureProfile{DataShards,ParityShards,...}     ErasureProfile(data_shards, parity_shards, shard_size)  metadata.go:4-8
    NewCodec()                                      Codec()                                                  codec.go:15-17
    (*Codec).Encode(data, profile)                  Codec.encode(data, profile) -> list of n shards          codec.go:21-41
    (*Codec).Decode(shards, profile, originalSize)  Codec.decode(shards, profile, original_size) -> bytes    codec.go:45-78
    ShardChecksum(data)                             shard_checksum(data)                                     codec.go:81-84
    ErrInsufficientShards/ErrShardCorrupted/...     exception classes of the same names                      errors.go:7-10

Go compares the sentinel errors by identity (codec_test.go:113,118); here each
sentinel is an exception class, and the wrapped upstream errors
("erasure: failed to split data: %w", codec.go:33 …) are raised as instances of the
upstream error's class carrying the wrapped message, so `isinstance` plays the role
of errors.Is and str() matches the Go .Error() text.

All shard arithmetic runs on the GPU through libcallfs_rs.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes
import hashlib
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N


# ---- errors (erasure/errors.go:7-10 and the upstream reedsolomon values) -------------

class ErasureError(Exception):
    """Base class for every error this module raises."""

    text = "erasure error"

    def __init__(self, message: Optional[str] = None):
        super().__init__(message if message is not None else self.text)


class ErrInsufficientShards(ErasureError):
    text = "erasure: insufficient shards for reconstruction (code 3050)"


class ErrShardCorrupted(ErasureError):
    text = "erasure: shard checksum mismatch (code 3051)"


class ErrInvalidProfile(ErasureError):
    text = "erasure: invalid erasure profile parameters (code 3054)"


class ErrShardNotFound(ErasureError):
    text = "erasure: shard not found on this node (code 3055)"


class ErrShortData(ErasureError):
    text = "not enough data to fill the number of requested shards"


class ErrTooFewShards(ErasureError):
    text = "too few shards given"


class ErrShardNoData(ErasureError):
    text = "no shard data"


class ErrShardSize(ErasureError):
    text = "shard sizes do not match"


class ErrSingular(ErasureError):
    text = "matrix is singular"


class ErrUnsupportedProfile(ErasureError):
    """k+m > 256: upstream reedsolomon.New switches to Leopard GF(2^16); the GPU codec
    does not implement it and the Go shim keeps the CPU codec for such profiles."""

    text = "profile needs the GF(2^16) (Leopard) codec: k+m > 256"


_UPSTREAM = {
    N.RS_E_SHORT_DATA: ErrShortData,
    N.RS_E_TOO_FEW_SHARDS: ErrTooFewShards,
    N.RS_E_SHARD_SIZE: ErrShardSize,
    N.RS_E_NO_DATA: ErrShardNoData,
    N.RS_E_SINGULAR: ErrSingular,
    N.RS_E_UNSUPPORTED: ErrUnsupportedProfile,
}


def _wrapped(rc: int, prefix: str) -> Exception:
    """fmt.Errorf(prefix + ": %w", upstreamErr)."""
    cls = _UPSTREAM.get(rc)
    if cls is None:
        return N.NativeError(rc, prefix)
    return cls(f"{prefix}: {cls.text}")


# ---- profile -----------------------------------------------------------------------

@dataclass
class ErasureProfile:
    """erasure/metadata.go:4-8."""

    data_shards: int
    parity_shards: int
    shard_size: int = 0


def shard_checksum(data) -> str:
    """codec.go:81-84: SHA-256 hex digest of a shard."""
    return hashlib.sha256(bytes(data)).hexdigest()


def shard_layout(data, shards) -> List[tuple]:
    """Where and under which checksum Manager.StoreFile keeps each shard
    (erasure/manager.go:171-184): path ".erasure/<first 8 bytes of SHA-256(object), hex>/<i>"
    and ShardChecksum(shard). The shard files are the raw shard bytes, so files written
    from this codec's shards are what the CPU codec reads back, and the reverse."""
    prefix = hashlib.sha256(bytes(data)).digest()[:8].hex()
    return [(f".erasure/{prefix}/{i}", shard_checksum(sh)) for i, sh in enumerate(shards)]


def _addr(buf) -> int:
    """Address of a bytes-like object's first byte (read-only objects allowed)."""
    a = np.frombuffer(buf, dtype=np.uint8)
    return a.ctypes.data if a.size else 0


def _writable(buf) -> bool:
    return isinstance(buf, (bytearray, np.ndarray)) or (
        isinstance(buf, memoryview) and not buf.readonly)


class Codec:
    """erasure/codec.go:12 Codec — stateless; one instance may be shared by threads
    like the shared *Codec at erasure/manager.go:60."""

    def __init__(self, context: Optional[N.Context] = None):
        self._ctx = context

    @property
    def context(self) -> N.Context:
        if self._ctx is None:
            self._ctx = N.default_context()
        return self._ctx

    def encode(self, data, profile: ErasureProfile) -> List[memoryview]:
        """codec.go:21-41. Returns data_shards+parity_shards equal-length shards: S =
        ceil(len/k); like upstream Split the full data shards are views into `data`
        (no copy), the shard holding the end of the object and any after it are
        zero-padded copies, and only the m parity shards are computed (rs_encode).
        Upstream Split also reuses a Go slice's spare capacity past len for the padded
        and parity shards; Python buffers expose no such capacity, so this mirror always
        allocates them (the Go shim, go/erasure/codec_rocm.go split, does reuse it)."""
        k, m = profile.data_shards, profile.parity_shards
        if k < 1 or m < 1:
            raise ErrInvalidProfile()
        src = memoryview(data).cast("B")
        L = len(src)
        # upstream New succeeds for k+m > 256 (Leopard GF(2^16)), so an empty object
        # still fails in Split first (codec.go:26 then :31)
        if L == 0:
            raise ErrShortData(f"erasure: failed to split data: {ErrShortData.text}")
        if k + m > 256:
            raise _wrapped(N.RS_E_UNSUPPORTED, "erasure: failed to create encoder")
        S = (L + k - 1) // k
        full = L // S  # data shards lying entirely inside `data`
        tail = bytearray(S * (k - full))
        tail[: L - full * S] = src[full * S:]
        parity = bytearray(S * m)
        tv, pv = memoryview(tail), memoryview(parity)
        shards = [src[i * S:(i + 1) * S] for i in range(full)]
        shards += [tv[i * S:(i + 1) * S] for i in range(k - full)]
        shards += [pv[j * S:(j + 1) * S] for j in range(m)]
        dptr = (ctypes.c_void_p * k)(*[_addr(s) for s in shards[:k]])
        pptr = (ctypes.c_void_p * m)(*[_addr(s) for s in shards[k:]])
        rc = N.lib.rs_encode(self.context.handle, k, m, S, dptr, pptr)
        if rc != N.RS_OK:
            raise _wrapped(rc, "erasure: failed to encode parity")
        return shards

    def decode(self, shards: List, profile: ErasureProfile, original_size: int) -> bytearray:
        """codec.go:45-78. `None` or empty entries are missing shards; they are
        reconstructed in place (the list is mutated, as Go mutates its [][]byte).
        Returns a fresh buffer of original_size bytes (Go: buf[:originalSize])."""
        k, m = profile.data_shards, profile.parity_shards
        if k < 1 or m < 1:
            raise ErrInvalidProfile()
        n = k + m
        if k + m > 256:
            raise _wrapped(N.RS_E_UNSUPPORTED, "erasure: failed to create decoder")
        if len(shards) != n:
            raise ErrTooFewShards(f"erasure: reconstruction failed: {ErrTooFewShards.text}")
        lens = (ctypes.c_size_t * n)()
        for i, s in enumerate(shards):
            lens[i] = 0 if s is None else len(s)
        S = next((lens[i] for i in range(n) if lens[i]), 0)
        bufs = list(shards)
        for i in range(n):
            if lens[i] == 0 and S:
                bufs[i] = bytearray(S)  # upstream Reconstruct allocates missing shards
        ptrs = (ctypes.c_void_p * n)(*[_addr(b) if b is not None and len(b) else 0
                                      for b in bufs])
        out = bytearray(max(int(original_size), 0))
        rc = N.lib.rs_codec_decode(self.context.handle, k, m, ptrs, lens,
                                   _addr(out) if out else None, int(original_size))
        # upstream Reconstruct (codec.go:55) has filled the nil entries before Verify
        # (:59) and the join-length check (:73) can fail, so ErrShardCorrupted and
        # ErrInsufficientShards leave them filled too (as the Go shim does)
        if rc in (N.RS_OK, N.RS_E_CORRUPT, N.RS_E_INSUFFICIENT):
            for i in range(n):
                if shards[i] is None or len(shards[i]) == 0:
                    shards[i] = bufs[i]
        if rc == N.RS_OK:
            return out
        if rc == N.RS_E_CORRUPT:
            raise ErrShardCorrupted()
        if rc == N.RS_E_INSUFFICIENT:
            raise ErrInsufficientShards()
        if rc == N.RS_E_INVALID_PROFILE:
            raise ErrInvalidProfile()
        if rc in (N.RS_E_TOO_FEW_SHARDS, N.RS_E_SHARD_SIZE, N.RS_E_NO_DATA, N.RS_E_SINGULAR):
            raise _wrapped(rc, "erasure: reconstruction failed")
        raise N.NativeError(rc, "erasure: decode")


# ---- reedsolomon.Encoder-level helpers over host shards -----------------------------

def _shard_ptrs(shards: Sequence) -> ctypes.Array:
    return (ctypes.c_void_p * len(shards))(*[_addr(s) if s is not None and len(s) else 0
                                             for s in shards])


def encode_shards(shards: List, k: int, m: int, context: Optional[N.Context] = None) -> None:
    """upstream enc.Encode(shards) (codec.go:36): fills shards[k:] in place. Parity
    entries must be writable buffers of the data shards' size."""
    ctx = context or N.default_context()
    if len(shards) != k + m:
        raise ErrTooFewShards()
    S = len(shards[0])
    if any(len(s) != S for s in shards):
        raise ErrShardSize()
    if not all(_writable(s) for s in shards[k:]):
        raise TypeError("parity shards must be writable")
    data = _shard_ptrs(shards[:k])
    par = _shard_ptrs(shards[k:])
    N.check(N.lib.rs_encode(ctx.handle, k, m, S, data, par), "rs_encode")


def reconstruct(shards: List, k: int, m: int, context: Optional[N.Context] = None) -> None:
    """upstream enc.Reconstruct(shards) (codec.go:55); missing entries are replaced."""
    ctx = context or N.default_context()
    n = k + m
    if len(shards) != n:
        raise ErrTooFewShards()
    lens = (ctypes.c_size_t * n)(*[0 if s is None else len(s) for s in shards])
    S = next((lens[i] for i in range(n) if lens[i]), 0)
    bufs = [bytearray(S) if (lens[i] == 0 and S) else shards[i] for i in range(n)]
    rc = N.lib.rs_reconstruct(ctx.handle, k, m, _shard_ptrs(bufs), lens)
    if rc != N.RS_OK:
        raise _wrapped(rc, "reconstruct")
    for i in range(n):
        if shards[i] is None or len(shards[i]) == 0:
            shards[i] = bufs[i]


def verify(shards: List, k: int, m: int, context: Optional[N.Context] = None) -> bool:
    """upstream enc.Verify(shards) (codec.go:59)."""
    ctx = context or N.default_context()
    n = k + m
    if len(shards) != n:
        raise ErrTooFewShards()
    lens = (ctypes.c_size_t * n)(*[0 if s is None else len(s) for s in shards])
    ok = ctypes.c_int(0)
    rc = N.lib.rs_verify(ctx.handle, k, m, _shard_ptrs(shards), lens, ctypes.byref(ok))
    if rc != N.RS_OK:
        raise _wrapped(rc, "verify")
    return bool(ok.value)


# ---- batched host calls (many independent stripes per native call) ----------------

def encode_batch(stripes: Sequence[Sequence], k: int, m: int,
                 context: Optional[N.Context] = None) -> Tuple[List[List[bytearray]], List[int]]:
    """rs_encode_batch: stripes[b] holds the k data shards of stripe b (equal length
    within a stripe; stripes may differ). Returns (parity[b] = m fresh shards, status[b])
    with status[b] one of RS_OK / RS_E_NO_DATA (empty shards)."""
    ctx = context or N.default_context()
    B = len(stripes)
    sizes = (ctypes.c_size_t * max(B, 1))()
    parity = []
    for b, st in enumerate(stripes):
        if len(st) != k:
            raise ErrTooFewShards()
        S = len(st[0])
        if any(len(s) != S for s in st):
            raise ErrShardSize()
        sizes[b] = S
        parity.append([bytearray(S) for _ in range(m)])
    data = _shard_ptrs([s for st in stripes for s in st] or [None])
    par = _shard_ptrs([p for ps in parity for p in ps] or [None])
    status = (ctypes.c_int * max(B, 1))()
    rc = N.lib.rs_encode_batch(ctx.handle, k, m, B, sizes, data, par, status)
    if rc not in (N.RS_OK, N.RS_E_NO_DATA):
        N.check(rc, "rs_encode_batch")
    return parity, list(status)[:B]


def reconstruct_batch(stripes: List[List], k: int, m: int, verify: bool = True,
                      context: Optional[N.Context] = None) -> List[int]:
    """rs_reconstruct_batch: stripes[b] is an n-list of shards (None / empty = missing),
    reconstructed in place like reconstruct(); with verify the present parity beyond the
    first k is re-checked per stripe. Returns status[b] (RS_OK, RS_E_CORRUPT,
    RS_E_TOO_FEW_SHARDS, RS_E_SHARD_SIZE, RS_E_NO_DATA, ...)."""
    ctx = context or N.default_context()
    n = k + m
    B = len(stripes)
    if any(len(st) != n for st in stripes):
        raise ErrTooFewShards()
    # missing entries get fresh buffers in a per-stripe copy (upstream Reconstruct
    # allocates them); the caller's lists change only for stripes that succeeded
    flat, lens, bufs = [], (ctypes.c_size_t * max(B * n, 1))(), []
    for b, st in enumerate(stripes):
        ln = [0 if s is None else len(s) for s in st]
        S = next((x for x in ln if x), 0)
        cp = list(st)
        for i in range(n):
            lens[b * n + i] = ln[i]
            if ln[i] == 0 and S:
                cp[i] = bytearray(S)
        bufs.append(cp)
        flat += cp
    status = (ctypes.c_int * max(B, 1))()
    rc = N.lib.rs_reconstruct_batch(ctx.handle, k, m, B, _shard_ptrs(flat or [None]), lens,
                                    int(verify), status)
    if rc < 0 and rc not in (N.RS_E_CORRUPT, N.RS_E_TOO_FEW_SHARDS, N.RS_E_SHARD_SIZE,
                             N.RS_E_NO_DATA):
        if not (rc == N.RS_E_ARG and any(s == N.RS_E_ARG for s in list(status)[:B])):
            N.check(rc, "rs_reconstruct_batch")
    out = list(status)[:B]
    for b, st in enumerate(stripes):
        if out[b] in (N.RS_OK, N.RS_E_CORRUPT):
            for i in range(n):
                if st[i] is None or len(st[i]) == 0:
                    st[i] = bufs[b][i]
    return out


# ---- host-side matrices (no device needed) ------------------------------------------

def encode_matrix(k: int, m: int) -> np.ndarray:
    """(k+m) x k systematic matrix E = V . inv(V[0:k]) (upstream buildMatrix)."""
    E = np.zeros((k + m, k), dtype=np.uint8)
    rc = N.lib.rs_encode_matrix(k, m, E.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    if rc == N.RS_E_INVALID_PROFILE:
        raise ErrInvalidProfile()
    N.check(rc, "rs_encode_matrix")
    return E


def decode_rows(k: int, m: int, present: Sequence[bool]):
    """(valid, missing, rows) as the fused decode kernel applies them."""
    n = k + m
    pr = np.array([1 if p else 0 for p in present], dtype=np.uint8)
    valid = (ctypes.c_int * k)()
    missing = (ctypes.c_int * n)()
    nm = ctypes.c_int(0)
    rows = np.zeros((n, k), dtype=np.uint8)
    u8 = ctypes.POINTER(ctypes.c_uint8)
    rc = N.lib.rs_decode_rows(k, m, pr.ctypes.data_as(u8), valid, missing, ctypes.byref(nm),
                              rows.ctypes.data_as(u8))
    if rc != N.RS_OK:
        raise _wrapped(rc, "decode_rows")
    return list(valid), list(missing)[:nm.value], rows[:nm.value]
