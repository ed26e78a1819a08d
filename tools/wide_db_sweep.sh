# Many-input R <= 4 profiles (K 14..24) on non-power-of-two pitches: every nibble and
# double-buffered triple order (tools/order_ab.py), to bound tile_order.hpp tri_rule_order's
# double-buffered branch for K > 12. Usage: bash tools/wide_db_sweep.sh <tag> [k,m,S ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-wide_db}"; shift; mkdir -p "$OUT"
shapes=("$@")
[ ${#shapes[@]} -eq 0 ] && shapes=(20,4,838861 24,4,699051 14,4,1198373 14,2,1198373 20,2,838861
  20,4,3355444 24,4,2796203 14,4,4793491 20,4,1048576 16,4,2097152)
for sh in "${shapes[@]}"; do
  IFS=, read k m S <<< "$sh"
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  timeout -k 10 300 python -u tools/order_ab.py --rounds 4 \
    --orders consecutive,g2,x32,q8,tri,tri-g2,tri-x32,tri-q8,tri-x8 \
    --shape $k,$m,$S,$B >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || exit $?
done
