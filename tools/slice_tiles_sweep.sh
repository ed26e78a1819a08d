# CALLFS_RS_MAX_TILES_PER_LAUNCH sweep through the production dispatch (tools/kbench).
# MTS="0 1073741824" (default): 0 = the built-in slicing rule, 1073741824 = one launch.
# Usage: bash tools/slice_tiles_sweep.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-slices}"; mkdir -p "$OUT"; : > "$OUT/summary.txt"
for shape in "10 4 6710887 256" "10 4 1048576 1024" "10 4 1048576 256" "16 4 4194304 64" "4 2 1048576 2048" "10 4 107374183 8"; do
  set -- $shape
  for mt in ${MTS:-0 1073741824}; do
    CALLFS_RS_MAX_TILES_PER_LAUNCH=$mt KB_KEEP="@none@" timeout -k 10 120 tools/kbench $1 $2 $3 $4 7 10 > "$OUT/kb_${mt}_$1_$2_$3_$4.log" 2>&1 || exit $?
    echo "$shape max_tiles=$mt $(grep 'prod dispatch' "$OUT/kb_${mt}_$1_$2_$3_$4.log" | awk '{print $NF}')" | tee -a "$OUT/summary.txt"
  done
done
