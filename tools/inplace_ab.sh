# In-place chunk pipeline (CALLFS_RS_INPLACE_PIPELINE=1) vs the staged H2D/kernel/D2H
# pipeline for calls above the small limit: GPU tests with it on, then e2e sweeps.
# Usage: bash tools/inplace_ab.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-inplace}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
CALLFS_RS_INPLACE_PIPELINE=1 CALLFS_RS_SMALL_MAX_BYTES=65536 timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_inplace.log" 2>&1 || { tail -30 "$OUT/pytest_inplace.log"; exit 1; }
tail -1 "$OUT/pytest_inplace.log"
O="$OUT/sweep.jsonl"
export CALLFS_E2E_ENCODER=1
for prof in "16 4 0,5,16,19" "4 2 1,4" "10 4 0,1,2,3"; do
  set -- $prof
  for L in 4194304 16777216 67108864; do
    for t in 1 8; do
      for mode in staged inplace; do
        echo "{\"mode\": \"$mode\"}" >> $O
        CALLFS_RS_INPLACE_PIPELINE=$([ $mode = inplace ] && echo 1 || echo 0) timeout -k 10 60 "$R/tools/e2e_native" $1 $2 $L $t 0.8 $3 >> $O || exit 1
      done
    done
  done
done
echo ok
