"""Register / scratch / occupancy guard for the production kernels (CPU, no GPU needed).

`callfs_amd/build.py` records the compiler's kernel-resource-usage remarks for every
kernel in `callfs_amd/kernel_resources.json`. The LDS kernel's speed depends on its
waves per SIMD: the 16-row instances fell from 4 to 3 waves (129
VGPRs) once the ragged tail moved into the kernel, which cost RS(10,16) ~10 points of
HBM bandwidth before anyone noticed. These checks make such a drift fail the CPU suite.
"""
import json
import os
import re

import pytest

from callfs_amd import build as nb


def _report():
    if nb._stale() or not os.path.exists(nb.RESOURCES):
        nb.build()
    with open(nb.RESOURCES) as fh:
        rep = json.load(fh)
    if rep.get("digest") != nb._digest():
        nb.build(force=True)
        with open(nb.RESOURCES) as fh:
            rep = json.load(fh)
    return rep


@pytest.fixture(scope="module")
def kernels():
    ks = _report()["kernels"]
    assert ks, "no kernel-resource remarks were recorded"
    return ks


def _policy(k):
    """The Policy<...> template arguments of a kernel's name."""
    return [x.strip() for x in re.search(r"Policy<([^>]*)>", k["name"]).group(1).split(",")]


def _lds(ks):
    """Production LDS-kernel instances (the NOMATH ceiling forms, Policy argument 10, are
    measurement kernels of rs_plan_launch_ceiling and excluded)."""
    return [k for k in ks if "rs_apply_lds<" in k["name"] and _policy(k)[9] != "true"]


def test_every_kernel_reported(kernels):
    names = [k["name"] for k in kernels]
    # 16 row counts of the default LDS kernel, 8 v_perm rows, the byte tails, SHA-256
    assert sum("rs_apply_lds<" in n for n in names) >= 16 + 8 * 4 + 8 + 8
    assert sum("rs_apply_vec<" in n for n in names) >= 8
    assert sum("rs_apply_bytes<" in n for n in names) == 16
    assert any("sha256" in n for n in names)


def test_no_scratch_or_spills(kernels):
    for k in kernels:
        assert k.get("scratch", 0) == 0, k["name"]
        # (SGPR spills go to VGPR lanes, not memory: the v_perm kernel's coefficient
        # tables at R = 4 spill a few, which is allowed)
        assert k.get("vgpr_spill", 0) == 0, k["name"]


def test_lds_kernel_occupancy(kernels):
    """R <= 4: 8 waves; R 5..8: at least 7 (6 for the realigning form, 5 for the triple
    loads); R 9..16
    (16-byte entries): 4 waves."""
    for k in _lds(kernels):
        r = int(re.search(r"rs_apply_lds<(\d+),", k["name"]).group(1))
        realign = _policy(k)[10] not in ("false", "0")
        triple = _policy(k)[14] == "2"  # triple loads: 12 more VGPRs, measured at 5 waves
        vpf = _policy(k)[13] not in ("0",)  # early compare loads: one uint4 per Verify row
        if realign and triple:  # realigning triples: 67 VGPRs at R <= 4, 94 at R 5..8
            want = 7 if r <= 4 else 5
        elif _policy(k)[14] == "3":  # double-buffered triples (R <= 4): 81-96 VGPRs
            want = 5
        elif triple and vpf:  # triples with early compares (R <= 4): 67-75 VGPRs
            want = 6
        else:
            want = 8 if r <= 4 else (6 if realign else 5 if triple else 7) if r <= 8 else 4
        assert k["waves_per_simd"] >= want, (k["name"], k["vgprs"], k["waves_per_simd"])
        if r > 8:
            assert k["vgprs"] + k.get("agprs", 0) <= 128, k["name"]


def test_wide_groups_use_sdwa_addresses(kernels):
    """The production R 9..16 policies carry the SDWA flag (12th Policy argument)."""
    wide = [k for k in _lds(kernels) if int(re.search(r"rs_apply_lds<(\d+),", k["name"]).group(1)) > 8]
    assert len(wide) >= 16
    for k in wide:
        assert _policy(k)[11] == "true", k["name"]  # Policy::SDWA
