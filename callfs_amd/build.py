"""Build libcallfs_rs.so (HIP kernels + C ABI) in-tree for gfx950.

`python callfs_amd/build.py` or `__graft_entry__.build()`. The shared library lands
next to this file so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcallfs_rs.so")
SOURCES = ["rs_kernels.hip", "sha256.hip", "rs_capi.cpp"]
HEADERS = ["rs_kernels.hpp", "rs_apply.hpp", "tile_order.hpp", "gf256.hpp", "copy_pool.hpp", "dispatch.hpp", "sha256.hpp", os.path.join("..", "..", "include", "callfs_rs.h")]
ARCH = os.environ.get("CALLFS_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


def _digest() -> str:
    h = hashlib.sha256(ARCH.encode())
    for f in SOURCES + HEADERS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stale() -> bool:
    """Content-hash check (mtimes are not reliable across repo snapshots)."""
    try:
        with open(LIB + ".sha256") as fh:
            return not os.path.exists(LIB) or fh.read().strip() != _digest()
    except OSError:
        return True


def build(force: bool = False, extra_flags=None) -> str:
    if not force and not _stale():
        return LIB
    objs = []
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
             "-Wno-unused-result", "-Wno-cuda-compat"] + list(extra_flags or [])
    for src in SOURCES:
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + ".o")
        cmd = [_hipcc(), *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd.insert(1, "-x")
            cmd.insert(2, "hip")
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = LIB + ".tmp"
    subprocess.run([_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp],
                   check=True)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    with open(LIB + ".sha256", "w") as fh:
        fh.write(_digest())
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
