# Triple loads vs the ring of three in every tile order with an instance, over shard
# sizes 1-32 MiB and few-input profiles (aligned StripeBatch pitch = S rounded to 256 B),
# interleaved in one process per shape (tools/order_ab.py); fits tile_order.hpp tri_rule /
# tri_order. Usage: bash tools/tri_sweep.sh <tag> [shape ...] (shape = k,m,S)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tri_sweep}"; shift; mkdir -p "$OUT"
shapes=("$@")
[ ${#shapes[@]} -eq 0 ] && shapes=(4,2,1048576 4,2,2097152 4,2,4194304 4,2,8388608 4,2,16777216 4,2,33554432 4,2,5592406
  6,3,1048576 6,3,2796203 6,3,4194304 6,3,8388608 6,3,11184811 6,3,16777216
  8,4,2097152 8,4,4194304 8,4,8388608 8,4,16777216 10,4,1048576 10,4,1677722 10,4,4194304 10,4,6710887 10,4,16777216
  12,4,1398102 12,4,5592406 12,4,16777216 8,8,2097152 8,8,8388608 10,8,1677722 10,8,6710887 16,4,1048576 16,4,4194304 16,4,16777216)
for sh in "${shapes[@]}"; do
  IFS=, read k m S <<< "$sh"
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  timeout -k 10 300 python -u tools/order_ab.py --rounds 4 \
    --orders consecutive,g2,q8,q16,x32,tri,tri-g2,tri-x32,tri-q8,tri-q16,tri-x8 \
    --shape $k,$m,$S,$B >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || exit $?
done
