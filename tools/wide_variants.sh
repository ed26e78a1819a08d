# Wide / many-input shapes: production dispatch against the existing tile-order and
# input-ring variants and the no-lookup ceiling. Usage: bash tools/wide_variants.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-wide}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_ORD=1 KB_RING=1 KB_KEEP="lds ord|lds ring|nomath g2"
for sh in 10,12 10,16 20,16 32,16 32,8 10,8; do
  k=${sh%,*}; m=${sh#*,}
  timeout -k 10 200 "$R/tools/kbench" $k $m 1048576 256 5 10 > "$OUT/kbench_${k}_${m}.log" 2>&1 || exit $?
  grep -vE "^RS|variant" "$OUT/kbench_${k}_${m}.log" | sed "s/^/RS($k,$m) /"
done
