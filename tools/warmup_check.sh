# Is the tuned bench faster because the tuning launches warm the GPU? Forced order, tuner
# off, at warmup 5 and 100, beside the driver's own command. Usage: bash tools/warmup_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-warmcheck}"; mkdir -p "$OUT"
j() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline_decode"]["frac"], d["encode_ms_median_min"], d["config"]["tile_order"])'; }
for i in 1 2; do
  CALLFS_RS_TILE_ORDER=consecutive timeout -k 10 200 python3 bench.py --cpu-seconds 0 --tune 0 --steps 20 --warmup 5 > "$OUT/c_w5_$i.log" 2>&1 || exit $?
  echo "consecutive tune0 w5 $i: $(j $OUT/c_w5_$i.log)"
  CALLFS_RS_TILE_ORDER=consecutive timeout -k 10 200 python3 bench.py --cpu-seconds 0 --tune 0 --steps 20 --warmup 100 > "$OUT/c_w100_$i.log" 2>&1 || exit $?
  echo "consecutive tune0 w100 $i: $(j $OUT/c_w100_$i.log)"
  timeout -k 10 200 python3 bench.py --cpu-seconds 0 --steps 20 --warmup 5 > "$OUT/drv_$i.log" 2>&1 || exit $?
  echo "driver cmd (tuned) $i: $(j $OUT/drv_$i.log)"
  timeout -k 10 200 python3 bench.py --cpu-seconds 0 --tune 0 --steps 20 --warmup 100 > "$OUT/rule_w100_$i.log" 2>&1 || exit $?
  echo "rule tune0 w100 $i: $(j $OUT/rule_w100_$i.log)"
done
