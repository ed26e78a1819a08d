# G8 (8 stripes interleaved) on long shards: the write-pattern probe (tools/write_pattern.hip)
# found it the best write order for 4 and 8 rows at every shard size; the ring of three in G8
# against the rule and the tuner's forms, and the read / write ceilings in G8.
# Usage: bash tools/g8_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-g8}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for s in 10,4,6710887,256,- 10,4,6710887,256,0+1+2+3 10,8,6710887,64,- 8,8,8388608,64,- \
         10,4,8388608,64,- 10,4,1048576,256,- 16,4,4194304,128,- 10,4,16777216,32,-; do
  A+=(--shape "$s,planar")
done
timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 \
  --orders consecutive,g2,g8,q8,x32,tri,tri-g2,tri-q8,tri-x32 "${A[@]}" > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
timeout -k 10 300 python3 -u tools/ceiling_orders.py --orders consecutive,g2,g8,q8,x32 \
  --shape 10,4,6710887,256,-,planar --shape 10,8,6710887,64,-,planar > "$O/ceil.jsonl" 2>&1 || exit $?
echo "ceil ok"
