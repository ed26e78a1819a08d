# GPU tests, then decode per erasure pattern at the bench shape and a short bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG="${1:-vp}"; OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/decode_sweep.py > "$OUT/decode_bench_shape.jsonl" 2>&1 || exit $?
cut -c60-200 "$OUT/decode_bench_shape.jsonl"
timeout -k 10 300 python3 tools/decode_sweep.py --shard-bytes 6710887 --stripes 256 > "$OUT/decode_cfg2.jsonl" 2>&1 || exit $?
cut -c60-200 "$OUT/decode_cfg2.jsonl"
timeout -k 10 300 python3 bench.py --cpu-seconds 0 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-120
