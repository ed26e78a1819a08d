# One-dispatch small path vs the staged path (CALLFS_RS_SMALL_MAX_BYTES=0), RS(16,4)
# encoder path + decode {0,5,16,19} and RS(4,2) {1,4}, 1 and 8 threads, host buffers.
# Usage: bash tools/small_path_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-smallpath}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; O="$OUT/sweep.jsonl"
export CALLFS_E2E_ENCODER=1
for prof in "16 4 0,5,16,19" "4 2 1,4"; do
  set -- $prof
  for L in ${SIZES:-4096 16384 65536 262144 1048576}; do
    for t in 1 8; do
      for mode in staged small; do
        lim=$([ $mode = staged ] && echo 0 || echo ${SMALL_LIM:-67108864})
        echo "{\"mode\": \"$mode\", \"small_max\": $lim}" >> $O
        CALLFS_RS_SMALL_MAX_BYTES=$lim timeout -k 10 60 "$R/tools/e2e_native" $1 $2 $L $t 0.6 $3 >> $O || exit 1
      done
    done
  done
done
echo ok
