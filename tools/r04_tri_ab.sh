# Round 4: triple loads in the realigning kernel (Split layout) and triple loads in Q8/Q16
# on large power-of-two-pitch shards, against the rule, interleaved in one process
# (tools/order_ab.py). Usage: bash tools/r04_tri_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-r04_tri_ab}"; mkdir -p "$OUT"
ab() { timeout -k 10 300 python -u tools/order_ab.py "$@" >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"; }
# Split layout (odd S, odd base): configs[1] shape and the r03 split shapes
ab --orders realign,realign-x32,realign-tri,realign-tri-x32 --rounds 4 \
   --shape 10,4,6710887,40,-,split --shape 4,2,1048577,600,-,split --shape 6,3,2796203,150,-,split \
   --shape 10,8,1048577,200,-,split --shape 12,4,5592406,48,-,split --shape 5,3,209716,2000,-,split \
   --shape 4,2,16777217,40,-,split || exit $?
# aligned power-of-two pitches above 8 MiB: triples in every order vs the nibble orders
ab --orders consecutive,q8,q16,tri,tri-q8,tri-q16,tri-x32 --rounds 4 \
   --shape 4,2,16777216,40 --shape 4,2,8388608,80 --shape 6,3,11184811,40 --shape 8,4,8388608,40 \
   --shape 8,8,8388608,30 --shape 10,4,16777216,18 --shape 4,4,33554432,16 || exit $?
