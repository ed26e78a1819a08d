# GPU tests, then the Split-layout rule (realigning kernel in X32 order) against the
# consecutive form, and the configs[1] Split-layout bench line. Usage: bash tools/r03_split_check.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-split}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
bash tools/gpu_tests.sh "$TAG" || exit $?
SHAPES="--shape 10,4,6710887,64,-,split --shape 10,4,1048577,256,-,split --shape 10,4,6710887,64,5,split --shape 4,2,1048577,512,-,split --shape 6,3,1048577,256,-,split --shape 10,8,1048577,256,-,split"
timeout -k 10 400 python3 -u tools/order_ab.py --orders realign,realign-x32 $SHAPES > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || exit $?
cat "$OUT/ab.jsonl"
timeout -k 10 400 python3 bench.py --split-layout --shard-bytes 6710887 --stripes 256 --cpu-seconds 0 --steps 20 > "$OUT/bench_split.log" 2>&1 || exit $?
tail -1 "$OUT/bench_split.log" | cut -c1-400
