# Bench-shape tile-order check on one box: the driver's command (tuner on, its choices
# logged) beside the tuner off under each forced order at 100 warm-up steps (steady
# state), alternated. Usage: bash tools/tune_bench_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tunecheck}"; mkdir -p "$OUT"
j() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline_decode"]["frac"], d["config"]["tile_order"])'; }
for i in 1 2 3; do
  CALLFS_RS_TUNE_LOG=1 timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > "$OUT/tuned_$i.log" 2>&1 || exit $?
  echo "driver cmd (tuned) $i: $(j $OUT/tuned_$i.log)"
  for o in consecutive g2; do
    CALLFS_RS_TILE_ORDER=$o timeout -k 10 200 python3 bench.py --cpu-seconds 0 --tune 0 --steps 20 --warmup 100 > "$OUT/${o}_$i.log" 2>&1 || exit $?
    echo "$o w100 $i: $(j $OUT/${o}_$i.log)"
  done
done
grep -h "rs_plan_tune" "$OUT"/tuned_*.log
