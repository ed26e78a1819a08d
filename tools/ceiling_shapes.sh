# Per-shape memory ceilings beside the production dispatch (tools/kbench: prod dispatch,
# the no-lookup LDS kernel in two tile orders, D2D copy), 5 rounds x 10 iterations.
# Usage: bash tools/ceiling_shapes.sh <tag> [shapes "k,m k,m ..."] [shard bytes]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-ceil}"; SHAPES="${2:-10,4 10,8 32,8 20,4 10,12 10,16 20,16 32,16 4,2}"
SB="${3:-1048576}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_KEEP="nomath|hipMemcpy"
for sh in $SHAPES; do
  k=${sh%,*}; m=${sh#*,}
  timeout -k 10 150 "$R/tools/kbench" $k $m $SB 256 5 10 > "$OUT/kbench_${k}_${m}.log" 2>&1 || exit $?
  grep -E "prod dispatch|nomath|hipMemcpy" "$OUT/kbench_${k}_${m}.log" | sed "s/^/RS($k,$m) /"
done
