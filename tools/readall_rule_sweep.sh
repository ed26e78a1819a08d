# The profile sweep's 33 cells in the layout CallFS produces (upstream Split of an io.ReadAll
# body: data shards at pitch S in the body, parity in 64-B AllocAligned buffers), encode and a
# two-data-shard decode (in place; FRESH=1: into fresh buffers, as upstream Reconstruct
# allocates them), rule against rs_plan_tune (tools/ceiling_sweep.py).
# Usage: [FRESH=1] bash tools/readall_rule_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-readall_rule}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,readall" --shape "$k,$m,$S,$B,0+1,readall")
  done
done
timeout -k 10 1300 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned --fresh "${FRESH:-0}" "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo "readall sweep ok"
