"""ctypes binding of libcallfs_rs.so (include/callfs_rs.h).

The shared library is the product: there is no Python or CPU fallback. Importing
this module without the built library raises ImportError naming the build command;
creating a context without a HIP device raises RuntimeError.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# CALLFS_RS_LIB names another build of the same ABI (the development tools' A/B build,
# callfs_amd/build.py --ab); the product is libcallfs_rs.so
LIB_PATH = os.environ.get("CALLFS_RS_LIB") or os.path.join(HERE, "libcallfs_rs.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `python callfs_amd/build.py` "
        "(hipcc --offload-arch=gfx950); the RS path has no CPU fallback")

# PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7, loaded by file
# name). Loading torch first lets our DT_NEEDED libamdhip64.so.7 bind to that copy, so
# the process has ONE HIP/HSA runtime; loading ours first would bring in /opt/rocm's
# copy beside torch's and the second runtime fails to initialise the device.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - plain C-ABI use without torch
    pass

lib = ctypes.CDLL(LIB_PATH)

RS_OK = 0
RS_E_INVALID_PROFILE = -1
RS_E_SHORT_DATA = -2
RS_E_TOO_FEW_SHARDS = -3
RS_E_SHARD_SIZE = -4
RS_E_NO_DATA = -5
RS_E_CORRUPT = -6
RS_E_INSUFFICIENT = -7
RS_E_UNSUPPORTED = -8
RS_E_HIP = -9
RS_E_ARG = -10
RS_E_SINGULAR = -11
RS_E_NOMEM = -12

_vp = ctypes.c_void_p
_u8p = ctypes.POINTER(ctypes.c_uint8)
_sz = ctypes.c_size_t
_i64 = ctypes.c_int64
_int = ctypes.c_int

# name -> (restype, argtypes); this table is also what tests check against the header.
SIGNATURES = {
    "rs_init": (_int, [ctypes.POINTER(_vp), ctypes.c_uint]),
    "rs_shutdown": (None, [_vp]),
    "rs_device_count": (_int, [_vp]),
    "rs_abi_version": (_int, []),
    "rs_strerror": (ctypes.c_char_p, [_int]),
    "rs_shard_size": (_int, [_int, _int, _i64, ctypes.POINTER(_i64)]),
    "rs_encode_matrix": (_int, [_int, _int, _u8p]),
    "rs_decode_rows": (_int, [_int, _int, _u8p, ctypes.POINTER(_int), ctypes.POINTER(_int),
                              ctypes.POINTER(_int), _u8p]),
    "rs_codec_encode": (_int, [_vp, _int, _int, _vp, _sz, _vp, _sz, ctypes.POINTER(_sz)]),
    "rs_codec_decode": (_int, [_vp, _int, _int, ctypes.POINTER(_vp), ctypes.POINTER(_sz), _vp,
                               _i64]),
    "rs_host_alloc": (_int, [_vp, _sz, ctypes.POINTER(_vp)]),
    "rs_host_free": (_int, [_vp, _vp]),
    "rs_encode": (_int, [_vp, _int, _int, _sz, ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
    "rs_reconstruct": (_int, [_vp, _int, _int, ctypes.POINTER(_vp), ctypes.POINTER(_sz)]),
    "rs_verify": (_int, [_vp, _int, _int, ctypes.POINTER(_vp), ctypes.POINTER(_sz),
                         ctypes.POINTER(_int)]),
    "rs_encode_batch": (_int, [_vp, _int, _int, _int, ctypes.POINTER(_sz), ctypes.POINTER(_vp),
                               ctypes.POINTER(_vp), ctypes.POINTER(_int)]),
    "rs_reconstruct_batch": (_int, [_vp, _int, _int, _int, ctypes.POINTER(_vp), ctypes.POINTER(_sz),
                                    _int, ctypes.POINTER(_int)]),
    "rs_plan_create": (_int, [_vp, _int, _int, _int, _sz, _int, _u8p, ctypes.POINTER(_vp),
                              ctypes.POINTER(_vp)]),
    "rs_plan_launch": (_int, [_vp, _vp]),
    "rs_plan_launch_timed": (_int, [_vp, _vp, _vp, _vp]),
    "rs_plan_status": (_int, [_vp, _vp, ctypes.POINTER(_int)]),
    "rs_plan_stripe_status": (_int, [_vp, _vp, ctypes.POINTER(_int)]),
    "rs_plan_bytes": (ctypes.c_uint64, [_vp]),
    "rs_plan_groups": (ctypes.c_int, [_vp]),
    "rs_plan_forms": (_int, [_vp, ctypes.POINTER(_int), _int]),
    "rs_tune_table_reset": (_int, [ctypes.c_char_p]),
    "rs_tune_table_entries": (_int, []),
    "rs_plan_launch_ceiling": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    "rs_plan_launch_ceiling_timed": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp, _vp]),
    "rs_plan_destroy": (None, [_vp]),
    "rs_plan_tune": (_int, [_vp, _vp, _int, ctypes.POINTER(_int), _int]),
    "rs_plan_set_orders": (_int, [_vp, ctypes.POINTER(_int), _int]),
    "rs_encode_dev": (_int, [_vp, _int, _int, _int, _sz, _int, ctypes.POINTER(_vp), _vp]),
    "rs_decode_dev": (_int, [_vp, _int, _int, _int, _sz, _int, _u8p, ctypes.POINTER(_vp), _vp]),
    "rs_sha256_plan_create": (_int, [_vp, _int, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_uint64),
                                     _int, ctypes.POINTER(_vp)]),
    "rs_sha256_plan_launch": (_int, [_vp, _vp, _vp]),
    "rs_sha256_plan_destroy": (None, [_vp]),
    "rs_sha256_dev": (_int, [_vp, _int, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_uint64), _int,
                             _vp, _vp]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


def strerror(code: int) -> str:
    return lib.rs_strerror(code).decode()


class NativeError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} (rc={code})" if what else strerror(code))


def check(rc: int, what: str = "") -> None:
    if rc != RS_OK:
        raise NativeError(rc, what)


class Context:
    """Owns one rs_ctx (rs_init/rs_shutdown). Thread-safe like the C context."""

    def __init__(self, device_mask: int = 0):
        h = _vp()
        rc = lib.rs_init(ctypes.byref(h), device_mask)
        if rc != RS_OK:
            raise RuntimeError(f"rs_init failed: {strerror(rc)} — the RS path needs a HIP "
                               "device (no CPU fallback)")
        self.handle = h

    @property
    def device_count(self) -> int:
        return lib.rs_device_count(self.handle)

    def close(self) -> None:
        if self.handle:
            lib.rs_shutdown(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedBuffer:
    """rs_host_alloc memory as a writable uint8 numpy array (`.array`). Host-memory calls
    whose buffers all lie in such allocations DMA them directly (no staging copy)."""

    def __init__(self, nbytes: int, context: "Context"):
        import numpy as np
        self.ctx = context
        p = _vp()
        check(lib.rs_host_alloc(context.handle, nbytes, ctypes.byref(p)), "rs_host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.ptr))

    def close(self) -> None:
        if getattr(self, "ptr", None):
            self.array = None
            check(lib.rs_host_free(self.ctx.handle, ctypes.c_void_p(self.ptr)), "rs_host_free")
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default = None
_default_lock = threading.Lock()


def default_context() -> Context:
    """Process-wide context over the devices in CALLFS_RS_DEVICE_MASK (0 = all)."""
    global _default
    with _default_lock:
        if _default is None:
            _default = Context(int(os.environ.get("CALLFS_RS_DEVICE_MASK", "0"), 0))
        return _default
