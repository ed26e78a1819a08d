"""ctypes binding of oracle/build/librs_oracle.so (the C oracle and CPU baseline).

TEST INFRASTRUCTURE ONLY (see oracle/rs_oracle.c header). Used by tests/ as a fast
checker for MiB-scale cases and by bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "librs_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        u8p = P(ctypes.c_uint8)
        L.orc_encode_matrix.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.orc_invert.argtypes = [ctypes.c_int, u8p, u8p]
        L.orc_apply_scalar.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t,
                                       P(ctypes.c_void_p), P(ctypes.c_void_p)]
        L.orc_apply_simd.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t,
                                     P(ctypes.c_void_p), P(ctypes.c_void_p), ctypes.c_int]
        L.orc_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                      P(ctypes.c_void_p), u8p]
        L.orc_verify.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, P(ctypes.c_void_p)]
        L.orc_simd_kind.restype = ctypes.c_int
        L.orc_bench_codec.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, u8p,
                                      ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, u8p,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                      P(ctypes.c_double), P(ctypes.c_int)]
        L.orc_bench_codec.restype = ctypes.c_int
        _lib = L
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def encode_matrix(k: int, m: int) -> np.ndarray:
    E = np.zeros((k + m, k), dtype=np.uint8)
    assert lib().orc_encode_matrix(k, m, _u8(E)) == 0
    return E


def apply(coef: np.ndarray, inputs, simd: bool = False, nthreads: int = 1):
    """out_r = XOR_i coef[r, i] * inputs[i]; inputs: list of equal-length uint8 arrays."""
    coef = np.ascontiguousarray(coef, dtype=np.uint8)
    rows, k = coef.shape
    S = len(inputs[0])
    outs = [np.empty(S, dtype=np.uint8) for _ in range(rows)]
    ins = [np.ascontiguousarray(x, dtype=np.uint8) for x in inputs]
    if simd:
        lib().orc_apply_simd(rows, k, _u8(coef), S, _ptrs(ins), _ptrs(outs), nthreads)
    else:
        lib().orc_apply_scalar(rows, k, _u8(coef), S, _ptrs(ins), _ptrs(outs))
    return outs


def encode(data_shards, k: int, m: int, simd: bool = False, nthreads: int = 1):
    E = encode_matrix(k, m)
    return apply(E[k:], data_shards, simd=simd, nthreads=nthreads)


def reconstruct(shards, present, k: int, m: int):
    """Fill missing shards (entries may be None); returns the list of n arrays."""
    S = next(len(s) for s in shards if s is not None)
    full = [np.ascontiguousarray(s, dtype=np.uint8) if s is not None else np.zeros(S, np.uint8)
            for s in shards]
    pr = np.array([1 if p else 0 for p in present], dtype=np.uint8)
    rc = lib().orc_reconstruct(k, m, S, _ptrs(full), _u8(pr))
    if rc != 0:
        raise ValueError(f"orc_reconstruct rc={rc}")
    return full


def verify(shards, k: int, m: int) -> bool:
    S = len(shards[0])
    arr = [np.ascontiguousarray(s, dtype=np.uint8) for s in shards]
    return bool(lib().orc_verify(k, m, S, _ptrs(arr)))


BENCH_ENCODE, BENCH_RECONSTRUCT, BENCH_VERIFY = 1, 2, 4
BENCH_MODES = {"stripe-parallel": 0, "byte-range": 1}


def bench_codec(buf: np.ndarray, k: int, m: int, S: int, present=None,
                ops: int = BENCH_ENCODE | BENCH_RECONSTRUCT | BENCH_VERIFY,
                mode: str = "stripe-parallel", nthreads: int = 1, seconds: float = 1.0):
    """Native timing loop of the reference's per-object work (rs_oracle.c
    orc_bench_codec) over buf = uint8 [stripes][k+m][pitch] (C-contiguous; shards are
    the first S bytes of each row). Erased shards (present[i] false) are reconstructed
    in place. Returns (verify_mismatches, elapsed_seconds, passes)."""
    assert buf.dtype == np.uint8 and buf.ndim == 3 and buf.flags.c_contiguous
    ns, n, pitch = buf.shape
    assert n == k + m and S <= pitch
    pr = None if present is None else np.array([1 if p else 0 for p in present], np.uint8)
    el, passes = ctypes.c_double(0), ctypes.c_int(0)
    rc = lib().orc_bench_codec(k, m, S, _u8(buf), n * pitch, pitch, ns,
                               None if pr is None else _u8(pr), ops, BENCH_MODES[mode],
                               nthreads, seconds, ctypes.byref(el), ctypes.byref(passes))
    if rc < 0:
        raise ValueError(f"orc_bench_codec rc={rc}")
    return rc, el.value, passes.value


def simd_kind() -> str:
    return {2: "gfni-avx512", 1: "avx2-pshufb", 0: "scalar"}[lib().orc_simd_kind()]
