# Shard layouts in HBM for the same workloads (tools/ceiling_sweep.py, rule and tuned):
# 'pitch' ([b][n][pitch]), 'planar' ([b][k][pitch] + [b][m][pitch]), 'shardmajor'
# ([n][b][pitch]); encode and decodes. Usage: bash tools/layout_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-lprobe}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for s in 10,4,1048576,256 10,4,104858,1024 8,4,2097152,128 4,2,16777216,32 10,4,6710887,64 6,3,174763,2048; do
  for e in - 0+1 5; do
    for L in pitch planar shardmajor; do A+=(--shape "$s,$e,$L"); done
  done
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo "sweep ok"
