# configs[1]/[2] on the current build: bench line at the 64 MiB-object shape, decode per
# erasure pattern at that shape and at the bench shape. Usage: bash tools/cfg12_r02.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG="${1:-cfg12}"; OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py --shard-bytes 6710887 --stripes 256 --steps 10 --warmup 2 --cpu-seconds 0 \
  > "$OUT/bench_cfg1.log" 2>&1 || exit $?
tail -1 "$OUT/bench_cfg1.log" | cut -c1-200
timeout -k 10 300 python3 tools/decode_sweep.py --shard-bytes 6710887 --stripes 256 > "$OUT/decode_cfg2.jsonl" 2>&1 || exit $?
cat "$OUT/decode_cfg2.jsonl" | cut -c1-200
timeout -k 10 300 python3 tools/decode_sweep.py > "$OUT/decode_bench_shape.jsonl" 2>&1 || exit $?
cat "$OUT/decode_bench_shape.jsonl" | cut -c1-200
