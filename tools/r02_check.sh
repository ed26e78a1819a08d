# Round-2 checks in one call: new GPU tests, realignment sweep, pinned-pool e2e probes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-r02c}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "host_pool or configs3 or cgo or chunk_shapes or pinned" > "$OUT/pytest_new.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_new.log"; [ $rc -eq 0 ] || exit $rc
bash tools/realign_sweep.sh "$TAG/realign" || exit $?
E="$R/tools/e2e_native"
export CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1
for t in 1 8; do
  echo "{\"case\": \"t${t}_fresh_pooled\"}" >> "$OUT/zc.jsonl"
  CALLFS_E2E_FRESH=1 timeout -k 10 120 $E 4 2 268435456 $t 6 1,4 >> "$OUT/zc.jsonl" 2>> "$OUT/zc.err" || exit $?
  tail -1 "$OUT/zc.jsonl"
done
