# The profile sweep's 33 cells (11 RS profiles x 1, 16, 64 MiB objects, ~4 GiB batches) in
# the 256-B-pitch layout with each stripe's shards in one block ('pitch') and with data and
# parity in two regions ('planar'), production rule and tuned (tools/ceiling_sweep.py, one
# process per pass, layouts alternated per cell). Usage: bash tools/layout_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-layout}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,pitch" --shape "$k,$m,$S,$B,-,planar")
  done
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo "sweep ok"
