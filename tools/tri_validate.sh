# Round 4: shapes outside the tri_sweep fit (other K, R and sizes), encode and read-only
# (download Verify), every order with an instance; then the one-erasure decode A/B.
# Usage: bash tools/tri_validate.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tri_validate}"; mkdir -p "$OUT"
for sh in 5,3,2097152 5,3,8388608 5,3,16777216 4,4,8388608 4,4,16777216 6,6,4194304 6,6,16777216 \
          4,1,16777216 9,3,16777216 8,4,33554432 6,3,33554432 4,2,67108864 5,2,3355444 10,6,16777216 \
          12,4,33554432 7,3,8388608; do
  IFS=, read k m S <<< "$sh"
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  timeout -k 10 300 python -u tools/order_ab.py --rounds 4 \
    --orders consecutive,g2,q8,q16,x32,tri,tri-g2,tri-x32,tri-q8,tri-q16 \
    --shape $k,$m,$S,$B >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || exit $?
done
for sh in 4,2,1048576 4,2,8388608 6,3,16777216 10,4,16777216 10,4,4194304 8,4,8388608; do
  IFS=, read k m S <<< "$sh"
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  timeout -k 10 300 python -u tools/order_ab.py --rounds 4 \
    --orders consecutive,q8,q16,x32,tri,tri-g2,tri-x32,tri-q8,tri-q16 \
    --shape $k,$m,$S,$B,none >> "$OUT/ab_readonly.jsonl" 2>> "$OUT/ab.err" || exit $?
done
