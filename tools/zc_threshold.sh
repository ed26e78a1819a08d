# Zero-copy threshold (CALLFS_RS_ZERO_COPY_MIN_BYTES, rs_capi.cpp zc_min) on the current
# build: rs_host_alloc buffers through the zero-copy launch (threshold 1 B) against the
# one-dispatch small path / staged pipeline (threshold 1 GiB), encode + decode, 1 and 8
# request threads. Output: gpurun_out/<tag>/zc.jsonl. Usage: bash tools/zc_threshold.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-zc_threshold}"; mkdir -p "$OUT"; O=$OUT/zc.jsonl; : > $O
for km in "16 4" "10 4" "4 2"; do
  set -- $km; k=$1; m=$2
  for L in 131072 262144 393216 524288 786432 1048576 1572864; do
    for th in 1 8; do
      for zc in 1 1073741824; do
        echo "{\"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th, \"zc_min\": $zc}" >> $O
        CALLFS_RS_ZERO_COPY_MIN_BYTES=$zc CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 \
          timeout -k 10 60 tools/e2e_native $k $m $L $th 0.5 0,$k >> $O || exit 1
      done
    done
  done
done
echo ok
