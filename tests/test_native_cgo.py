"""tests/native/cgo_drive.c: the C ABI driven the way the cgo shim drives it
(C-malloc'd pointer and lens arrays, nil entries as lens 0), every Decode error path
leaving lens and the missing buffers untouched. CPU: AddressSanitizer + UBSan build of
the driver, argument paths only (no device). GPU: plain build, plus round trips
against the C oracle."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "cgo_drive.c")


def _build(out, sanitize):
    from oracle import cref
    cref.build()
    flags = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"] if sanitize else []
    subprocess.run(["gcc", "-std=c11", "-O1", *flags, "-I", os.path.join(ROOT, "include"), SRC,
                    "-o", str(out), "-L", os.path.join(ROOT, "callfs_amd"), "-lcallfs_rs",
                    "-L", os.path.join(ROOT, "oracle", "build"), "-lrs_oracle",
                    "-Wl,-rpath," + os.path.join(ROOT, "callfs_amd"),
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle", "build")], check=True)


def test_cgo_argument_paths_asan(tmp_path, native_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu variant")
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = tmp_path / "cgo_drive_asan"
    _build(exe, sanitize=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cgo_drive ok (argument paths" in r.stdout


@pytest.mark.gpu
def test_cgo_drive_device(tmp_path, native_lib):
    exe = tmp_path / "cgo_drive"
    _build(exe, sanitize=False)
    r = subprocess.run([str(exe), "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cgo_drive ok (device round trips)" in r.stdout
