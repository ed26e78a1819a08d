"""Host-side C++ of the RS path (GF math, v_perm table packing, decode rows, copy pool)
built with g++ under AddressSanitizer+UBSan and ThreadSanitizer and run on the CPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "host_test.cpp")
INC = os.path.join(ROOT, "callfs_amd", "csrc")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_host_code_under_sanitizer(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = tmp_path / f"host_test_{san.split(',')[0]}"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}",
                    "-fno-omit-frame-pointer", "-I", INC, SRC, "-o", str(exe), "-lpthread"],
                   check=True)
    env = dict(os.environ, CALLFS_RS_COPY_THREADS="4")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_test ok" in r.stdout


def test_bitslice_kernels_compile_for_gfx950(tmp_path):
    """The bit-sliced kernels' generated sources compile with hiprtc for gfx950 on the CPU
    (no GPU): encode blocks of 9, 16 and 8 rows over 10 to 64 inputs, K > 32 included (a
    generator that shadowed a helper with shard 32's buffer compiled nothing above 32), and
    the occupancy search ends with at most 16 spilled VGPRs."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = tmp_path / "bs_compile"
    subprocess.run([hipcc, "-O1", "-std=c++17", "-x", "hip", "--offload-arch=gfx950", "-I", INC,
                    os.path.join(ROOT, "tests", "native", "bs_compile.cpp"),
                    os.path.join(INC, "bitslice.cpp"), "-lhiprtc", "-o", str(exe)],
                   check=True, capture_output=True)
    env = dict(os.environ, CALLFS_RS_JIT_CACHE="0", CALLFS_OFFLOAD_ARCH="gfx950")
    r = subprocess.run([str(exe), "10,9", "20,16", "33,12", "64,8"], capture_output=True,
                       text=True, env=env, timeout=600)
    assert r.returncode == 0 and "bs_compile ok" in r.stdout, r.stdout + r.stderr[-2000:]


def test_bitslice_code_object_cache(tmp_path):
    """The on-disk code-object cache (CALLFS_RS_JIT_CACHE): a second process loads the entry
    the first wrote (same waves floor and spills; an edited header field shows the entry, not
    a compile, was used), and a damaged entry is a miss that is compiled and rewritten."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = tmp_path / "bs_compile"
    subprocess.run([hipcc, "-O1", "-std=c++17", "-x", "hip", "--offload-arch=gfx950", "-I", INC,
                    os.path.join(ROOT, "tests", "native", "bs_compile.cpp"),
                    os.path.join(INC, "bitslice.cpp"), "-lhiprtc", "-o", str(exe)],
                   check=True, capture_output=True)
    cache = tmp_path / "cache"
    env = dict(os.environ, CALLFS_RS_JIT_CACHE=str(cache), CALLFS_OFFLOAD_ARCH="gfx950")

    def run():
        r = subprocess.run([str(exe), "20,16"], capture_output=True, text=True, env=env,
                           timeout=600)
        assert r.returncode == 0 and "bs_compile ok" in r.stdout, r.stdout + r.stderr[-2000:]
        line = r.stdout.splitlines()[0]
        fields = dict(f.split("=") for f in line.split() if "=" in f)
        return fields["waves"], fields["spills"], float(line.split()[-2])

    w1, s1, _ = run()
    entries = [p for p in cache.iterdir() if p.suffix == ".co"]
    assert len(entries) == 1, entries
    blob = entries[0].read_bytes()
    assert blob[:4] == b"CFBS" and blob[16:20] == b"\x7fELF"
    w2, s2, _ = run()
    assert (w2, s2) == (w1, s1), (w1, s1, w2, s2)
    # the second process read the entry, not the compiler: a waves field edited in the file's
    # header is what it reports
    import struct
    edited = blob[:4] + struct.pack("<i", 7) + blob[8:]
    entries[0].write_bytes(edited)
    w2b, _, _ = run()
    assert w2b == "7", w2b
    entries[0].write_bytes(blob[:len(blob) // 2])  # truncated: a miss, compiled again
    w3, s3, _ = run()
    assert (w3, s3) == (w1, s1)
    assert entries[0].read_bytes() == blob


def test_bitslice_compile_worker_under_tsan(tmp_path):
    """The bit-sliced kernels' compile state machine (bitslice.cpp Kernel / Worker /
    kernel_for) from eight threads under ThreadSanitizer, hiprtc compiling on the CPU: every
    kernel ends Ready once, one Kernel per coefficient block, and a background compile still
    queued or running at exit neither crashes nor races comgr's teardown (round 6 found the
    worker compiling while comgr's static destructors ran: SIGSEGV or a double free at exit)."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = tmp_path / "bs_worker"
    subprocess.run([hipcc, "-O1", "-g", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                    "-Xarch_host", "-fsanitize=thread", "-I", INC,
                    os.path.join(ROOT, "tests", "native", "bs_worker.cpp"),
                    os.path.join(INC, "bitslice.cpp"), "-lhiprtc", "-o", str(exe)],
                   check=True, capture_output=True)
    env = dict(os.environ, CALLFS_RS_JIT_CACHE="0", CALLFS_OFFLOAD_ARCH="gfx950")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0 and "bs_worker ok" in r.stdout, r.stdout + r.stderr[-3000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
