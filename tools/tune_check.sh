# rs_plan_tune on the bench workload: three bench runs with the tuner's per-order times
# logged, interleaved with runs on the rule's order (--tune 0). Usage: bash tools/tune_check.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-tune}"; shift
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
export CALLFS_RS_TUNE_LOG=1
for i in 1 2 3; do
  for t in 1 0; do
    timeout -k 10 300 python3 bench.py --cpu-seconds 0 --ceiling 0 --tune $t "$@" > "$OUT/bench_${i}_tune$t.log" 2>&1 || exit $?
    echo "run $i tune=$t: $(grep rs_plan_tune "$OUT/bench_${i}_tune$t.log" | tr '\n' ' ')"
    tail -1 "$OUT/bench_${i}_tune$t.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  value', d['value'], 'enc', d['roofline']['frac'], 'dec', d['roofline_decode']['frac'], d['config']['tile_order'])"
  done
done
