"""Build libcallfs_rs.so (HIP kernels + C ABI) in-tree for gfx950.

`python callfs_amd/build.py` or `__graft_entry__.build()`. The shared library lands
next to this file so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures
import hashlib
import json
import os
import subprocess
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcallfs_rs.so")
# The A/B build (rs_kernels.hpp CALLFS_RS_AB_INSTANCES): the product plus the measurement-only
# kernel forms and toggles, for the development tools (CALLFS_RS_LIB=<this path>). Built on
# demand (`python callfs_amd/build.py --ab`, the probe scripts run it on the GPU box) into
# build/ab/, outside the package: gpurun pushes and the round-end runs carry only the product.
LIB_AB = os.path.join(os.path.dirname(HERE), "build", "ab", "libcallfs_rs_ab.so")
# Per-kernel register / scratch / occupancy report of the last build (the compiler's
# kernel-resource-usage remarks), checked by tests/test_kernel_resources.py: the LDS
# kernel's speed depends on its waves per SIMD.
RESOURCES = os.path.join(HERE, "kernel_resources.json")
SOURCES = ["rs_kernels.hip", "sha256.hip", "rs_capi.cpp", "bitslice.cpp"]
HEADERS = ["bitslice.hpp", "bitslice_gen.hpp", "bitslice_rule.hpp", "tune_table.hpp", "rs_kernels.hpp", "rs_apply.hpp", "tile_order.hpp", "gf256.hpp", "copy_pool.hpp", "dispatch.hpp", "sha256.hpp", os.path.join("..", "..", "include", "callfs_rs.h")]
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


def _stale(lib: str = LIB) -> bool:
    """Content-hash check (mtimes are not reliable across repo snapshots)."""
    try:
        with open(lib + ".sha256") as fh:
            return not os.path.exists(lib) or fh.read().strip() != _digest()
    except OSError:
        return True


def build(force: bool = False, extra_flags=None, ab: bool = False) -> str:
    """Builds libcallfs_rs.so (ab=False) or the A/B build libcallfs_rs_ab.so (ab=True)."""
    lib = LIB_AB if ab else LIB
    if not force and not _stale(lib):
        return lib
    objs = []
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
             "-Wno-unused-result", "-Wno-cuda-compat"] + list(extra_flags or [])
    if ab:
        flags.append("-DCALLFS_RS_AB_INSTANCES=1")
    kernels = []

    def compile_one(src):
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + (".ab.o" if ab else ".o"))
        cmd = [_hipcc(), *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd.insert(1, "-x")
            cmd.insert(2, "hip")
        else:
            cmd.append("-Rpass-analysis=kernel-resource-usage")
        return src, obj, cmd, subprocess.run(cmd, stderr=subprocess.PIPE, text=True)

    # the sources compile independently: in parallel (rs_kernels.hip dominates). A line on
    # stderr every 30 s: a GPU-box command that prints nothing for 3 minutes counts as hung
    done = threading.Event()

    def heartbeat():
        t0 = time.time()
        while not done.wait(30):
            sys.stderr.write(f"build.py: compiling {os.path.basename(lib)}, {time.time() - t0:.0f} s\n")
            sys.stderr.flush()

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        with concurrent.futures.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
            results = list(ex.map(compile_one, SOURCES))
    finally:
        done.set()
    for src, obj, cmd, r in results:
        kernels += _parse_resource_remarks(r.stderr)
        other = [ln for ln in r.stderr.splitlines() if "kernel-resource-usage" not in ln]
        if r.returncode != 0 or any("error" in ln or "warning" in ln for ln in other):
            sys.stderr.write("\n".join(other) + "\n")
        if r.returncode != 0:
            raise subprocess.CalledProcessError(r.returncode, cmd)
        objs.append(obj)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    tmp = lib + ".tmp"
    # libhiprtc: the bit-sliced kernels are compiled at plan time (csrc/bitslice.cpp)
    subprocess.run([_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-lhiprtc",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", tmp], check=True)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    if not ab:
        with open(RESOURCES, "w") as fh:
            json.dump({"digest": _digest(), "arch": ARCH, "instances": len(kernels),
                       "library_bytes": os.path.getsize(lib), "kernels": kernels}, fh, indent=1)
            fh.write("\n")
    with open(lib + ".sha256", "w") as fh:
        fh.write(_digest())
    return lib


def _parse_resource_remarks(text: str) -> list:
    """Kernel name, VGPRs, scratch bytes per lane, spills and occupancy from the
    `-Rpass-analysis=kernel-resource-usage` remarks hipcc prints per kernel."""
    out, cur = [], None
    keys = {"VGPRs": "vgprs", "AGPRs": "agprs", "ScratchSize [bytes/lane]": "scratch",
            "Occupancy [waves/SIMD]": "waves_per_simd", "VGPRs Spill": "vgpr_spill",
            "SGPRs Spill": "sgpr_spill", "TotalSGPRs": "sgprs"}
    for ln in text.splitlines():
        if "remark:" not in ln or "kernel-resource-usage" not in ln:
            continue
        body = ln.split("remark:", 1)[1].rsplit("[-Rpass", 1)[0].strip()
        if body.startswith("Function Name:"):
            cur = {"symbol": body.split(":", 1)[1].strip()}
            out.append(cur)
        elif cur is not None and ":" in body:
            k, v = body.rsplit(":", 1)
            if k.strip() in keys:
                try:
                    cur[keys[k.strip()]] = int(v.strip())
                except ValueError:
                    pass
    names = _demangle([k["symbol"] for k in out])
    for k, n in zip(out, names):
        k["name"] = n
    return out


def _demangle(symbols: list) -> list:
    try:
        r = subprocess.run(["c++filt"], input="\n".join(symbols), capture_output=True,
                           text=True, check=True)
        names = r.stdout.splitlines()
        if len(names) == len(symbols):
            return names
    except (OSError, subprocess.CalledProcessError):
        pass
    return list(symbols)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, ab="--ab" in sys.argv))
