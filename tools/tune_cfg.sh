# rs_plan_tune against the rule on configs[1]/[2] and the bench shape: encode and decode
# plans per erasure pattern, rule and tuned plan timed interleaved in one process.
# Usage: bash tools/tune_cfg.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG="${1:-tunecfg}"; OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
export CALLFS_RS_TUNE_LOG=1
P="enc;;5;0,3,7,12;0,1,2,3"
timeout -k 10 300 python3 tools/decode_sweep.py --tune 1 --patterns "$P" > "$OUT/bench_shape.jsonl" 2> "$OUT/bench_shape.err" || exit $?
cut -c1-260 "$OUT/bench_shape.jsonl"
timeout -k 10 400 python3 tools/decode_sweep.py --tune 1 --patterns "$P" --shard-bytes 6710887 --stripes 128 > "$OUT/cfg2.jsonl" 2> "$OUT/cfg2.err" || exit $?
cut -c1-260 "$OUT/cfg2.jsonl"
timeout -k 10 300 python3 tools/decode_sweep.py --tune 1 --patterns "enc" --k 4 --m 2 --stripes 1024 > "$OUT/rs4_2.jsonl" 2> "$OUT/rs4_2.err" || exit $?
cut -c1-260 "$OUT/rs4_2.jsonl"
timeout -k 10 300 python3 tools/decode_sweep.py --tune 1 --patterns "enc" --k 16 --m 4 --shard-bytes 4194304 --stripes 64 > "$OUT/rs16_4_4m.jsonl" 2> "$OUT/rs16_4_4m.err" || exit $?
cut -c1-260 "$OUT/rs16_4_4m.jsonl"
timeout -k 10 300 python3 tools/decode_sweep.py --tune 1 --patterns "enc" --k 3 --m 2 --shard-bytes 349526 --stripes 1024 > "$OUT/rs3_2.jsonl" 2> "$OUT/rs3_2.err" || exit $?
cut -c1-260 "$OUT/rs3_2.jsonl"
