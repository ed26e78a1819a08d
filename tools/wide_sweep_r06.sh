# Wide and many-input profiles (the bit-sliced kernels' launches) at 1, 16 and 64 MiB
# objects, ~4 GiB batches, planar: production rule against rs_plan_tune (which also times
# the nibble-table forms). Usage: bash tools/wide_sweep_r06.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-wide}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "10 16" "20 16" "32 16" "16 8" "24 12" "20 9"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,planar")
  done
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo ok
