# Double-buffered triples (the "tri*" orders of R <= 4 launches with K >= 6) on many-input
# profiles beyond the rule's K <= 12 and on 1 MiB-object shards, against the nibble orders
# (tools/order_ab.py). Usage: bash tools/tridb_wide.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tridb_wide}"; mkdir -p "$OUT"
for sh in 16,4,1048576 16,4,4194304 16,4,65536 20,4,1048576 20,4,52429 24,4,1048576 32,4,1048576 32,4,32768 \
          14,2,1048576 20,2,1048576 10,4,104858 12,4,87382 10,2,104858 10,4,4194304 10,4,6710887 12,4,5592406 8,4,8388608; do
  IFS=, read k m S <<< "$sh"
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  timeout -k 10 300 python -u tools/order_ab.py --rounds 4 \
    --orders consecutive,g2,g8,x32,tri,tri-g2,tri-x32,tri-q8 \
    --shape $k,$m,$S,$B >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || exit $?
done
