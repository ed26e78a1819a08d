# Round-3 GPU pass: tests, small-path trace and sweep, LDS rate, decode / split ceilings,
# bench default and --split-layout (configs[1]). Usage: bash tools/r03_check.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-r03}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
[ -z "$SKIP_TESTS" ] && { bash tools/gpu_tests.sh "$TAG" || exit $?; }
[ -z "$SKIP_SMALL" ] && { bash tools/small_trace.sh "${TAG}_trace" || exit $?; }
[ -z "$SKIP_SMALL" ] && { SIZES="4096 65536" bash tools/small_path_sweep.sh "${TAG}_small" || exit $?; }
timeout -k 10 120 tools/lds_rate 4000 > "$OUT/lds_rate.txt" 2>&1; echo "lds_rate rc=$?"
timeout -k 10 300 python3 -u tools/ceiling_sweep.py --tune 1 \
  --shape 10,4,1048576,256,5 --shape 10,4,1048576,256,0 --shape 10,4,1048576,256,13 \
  --shape 10,4,6710887,64,5 --shape 10,4,6710887,64,0 --shape 10,4,6710887,64,13 \
  --shape 10,4,6710887,64,none --shape 10,4,6710887,64,0+3+7+12 \
  > "$OUT/decode.jsonl" 2> "$OUT/decode.err" || exit $?
echo decode ok
timeout -k 10 400 python3 bench.py > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 400 python3 bench.py --split-layout --shard-bytes 6710887 --stripes 256 --cpu-seconds 0 --steps 20 > "$OUT/bench_split.log" 2>&1 || exit $?
tail -1 "$OUT/bench_split.log" | cut -c1-300
timeout -k 10 400 python3 bench.py --shard-bytes 6710887 --stripes 256 --cpu-seconds 0 --steps 20 > "$OUT/bench_cfg1.log" 2>&1 || exit $?
tail -1 "$OUT/bench_cfg1.log" | cut -c1-300
