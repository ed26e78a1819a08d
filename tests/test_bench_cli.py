"""bench.py's launch contract on the CPU (no GPU work): --gpus N must equal the number
of ranks torch.distributed.run started (WORLD_SIZE), so a bare `--gpus 8` fails loudly
instead of printing a one-rank line."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_must_match_world_size():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr and "--nproc-per-node 8" in r.stderr


def test_load_traffic_matches_config_exactly(tmp_path):
    sys.path.insert(0, ROOT)
    import json
    import bench
    cfg = {"k": 10, "m": 4, "shard_bytes": 1 << 20, "stripes": 256, "erase": [0, 1, 2, 3]}
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"config": cfg, "encode_bytes_per_launch": 5, "decode_bytes_per_launch": 6}))
    assert bench.load_traffic(str(p), cfg)[:2] == (5, 6)
    assert bench.load_traffic(str(p), {**cfg, "stripes": 128}) == (None, None, None)
    assert bench.load_traffic(str(tmp_path / "missing.json"), cfg) == (None, None, None)


def test_committed_traffic_matches_the_default_bench_config():
    """profiles/hbm_traffic.json (the rocprofv3 PMC bytes the line quotes as `traffic`)
    is keyed by the default bench config, layout included."""
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse_args([])
    cfg = {"k": a.k, "m": a.m, "shard_bytes": a.shard_bytes, "stripes": 256}
    if a.layout != "pitch":
        cfg["layout"] = a.layout
    erase = sorted(int(x) for x in a.erase.split(","))
    enc, dec, src = bench.load_traffic(a.traffic, {**cfg, "erase": erase})
    assert enc and dec and src == os.path.join("profiles", "hbm_traffic.json")



@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--decode-into", "inplace"], ["--layout", "pitch"],
                                   ["--split-layout", "readall", "--shard-bytes", "100003"],
                                   ["--split-layout", "--shard-bytes", "100003"],
                                   ["--pitch", str((1 << 20) + 4096)],
                                   ["--object-bytes", str(16 << 20)]])
def test_bench_layouts_run_and_check(extra):
    """bench.py end to end on a small batch in every layout it offers: the device round
    trip, the timed steps, the rebuilt-shard check, the ceilings and (planar) the
    in-process pitch / readall layout A/B all pass, and the line parses."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stripes", "8",
                        "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.5",
                        "--cpu-working-set", str(64 << 20)] + extra,
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    assert line["cpu_baseline"]["parity_check"].startswith("GPU parity")
    if not extra:
        assert line["config"]["layout"] == "planar"
        ab = line["layout_ab"]
        assert "error" not in ab, ab
        for lay in ("pitch", "readall", "planar"):
            assert 0 < ab[lay]["encode_frac"] < 1 and 0 < ab[lay]["decode_frac"] < 1, lay
