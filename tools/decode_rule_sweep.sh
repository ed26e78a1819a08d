# Download-side launches on the planar layout, rule against rs_plan_tune: nothing erased
# (Verify only, read-only), one data shard lost (one written row + compared rows), two lost,
# and one parity lost (tools/ceiling_sweep.py, in place). Usage: bash tools/decode_rule_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-decrule}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "4 2" "6 3" "8 4" "10 4" "12 4" "16 4" "10 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,none,planar" --shape "$k,$m,$S,$B,1,planar" --shape "$k,$m,$S,$B,0+1,planar" --shape "$k,$m,$S,$B,$k,planar")
  done
done
timeout -k 10 1100 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo "decode sweep ok"
