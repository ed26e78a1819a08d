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
