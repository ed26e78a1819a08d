# Production dispatch (encode) over common RS profiles and object sizes, % of 8 TB/s.
# Usage: bash tools/profile_sweep.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-profiles}"; mkdir -p "$OUT"
: > "$OUT/summary.txt"
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do  # object bytes
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    KB_KEEP="@none@" timeout -k 10 120 tools/kbench $k $m $S $B 5 10 > "$OUT/kb_${k}_${m}_$L.log" 2>&1 || exit $?
    echo "RS($k,$m) object $L S=$S B=$B $(grep 'prod dispatch' "$OUT/kb_${k}_${m}_$L.log" | awk '{print $(NF-1), $NF}')" | tee -a "$OUT/summary.txt"
  done
done
