# The profile sweep's 33 cells (11 RS profiles x 1, 16, 64 MiB objects, ~4 GiB batches) in
# the planar layout (the bench layout), production rule against rs_plan_tune, two passes
# (tools/ceiling_sweep.py): the data the tile-order rule is fitted to (tile_order.hpp).
# Usage: [PASSES=n] bash tools/rule_sweep.sh <tag> [extra ceiling_sweep args]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-rule}"; shift; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,planar")
  done
done
for pass in $(seq 1 "${PASSES:-2}"); do
  timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
    > "$O/sweep_$pass.jsonl" 2>&1 || exit $?
  echo "pass $pass ok"
done
