# configs[3] per-rank shapes: 1 GiB RS(10,4) objects split by byte columns over N GPUs
# (callfs_amd/sharding.py column_slices) -> shard slice widths for N = 1, 2, 4, 8, each
# with ~6 GiB resident. Tile-order variants of the LDS kernel. Usage: bash tools/slice_sweep.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-slice}"; mkdir -p "$OUT"
for shape in "107374183 4" "53687296 8" "26843648 16" "13421824 32" "16777216 32" "1048576 256"; do
  set -- $shape
  KB_ORD=1 timeout -k 10 120 tools/kbench 10 4 $1 $2 5 10 > "$OUT/kb_10_4_$1_$2.log" 2>&1 || exit $?
  echo "== S=$1 B=$2"; cat "$OUT/kb_10_4_$1_$2.log" | tail -16
done
