# (round 2: spin polling measured no faster than hipEventSynchronize -- 28 us per 4 KiB call
#  either way -- and the CALLFS_RS_WAIT knob was removed; profiles/r02/small_latency/ keeps the data)
# Small-object round trip: hipEventSynchronize vs spin polling (CALLFS_RS_WAIT=spin),
# RS(16,4) encoder path + decode, staged and zero-copy, 1 thread. Usage: bash tools/small_latency.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-small}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; O="$OUT/small.jsonl"
for L in 4096 65536 1048576; do
  for w in sync spin; do
    for mode in staged pinned; do
      echo "{\"wait\": \"$w\", \"mode\": \"$mode\"}" >> $O
      env CALLFS_RS_WAIT=$w CALLFS_E2E_ENCODER=1 $([ $mode = pinned ] && echo CALLFS_E2E_PINNED=1) \
        timeout -k 10 60 "$R/tools/e2e_native" 16 4 $L 1 1.5 0,5,16,19 >> $O || exit 1
      tail -1 $O | cut -c1-220
    done
  done
done
