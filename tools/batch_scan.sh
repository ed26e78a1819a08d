# bench.py over batch sizes (stripes per GPU): per-launch kernel time vs batch separates
# the launch's fixed ramp-up / tail from its steady-state rate. Usage: bash tools/batch_scan.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-batch}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
for B in 64 128 256 512 1024; do
  timeout -k 10 200 python3 bench.py --stripes $B --cpu-seconds 0 --ceiling 0 --steps 30 > "$OUT/b$B.log" 2>&1 || exit $?
  python3 - "$OUT/b$B.log" $B <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], d["value"], d["encode_ms"], d["decode_ms"], d["launch_gap_ms"], d["config"]["tile_order"])
PY
done
