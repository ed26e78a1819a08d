"""bench.py's launch contract on the CPU (no GPU work): --gpus N must equal the number
of ranks torch.distributed.run started (WORLD_SIZE), so a bare `--gpus 8` fails loudly
instead of printing a one-rank line."""
import os
import subprocess
import sys

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
