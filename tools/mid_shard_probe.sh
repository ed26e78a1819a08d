# R <= 4, K >= 7, shards of 1-8 MiB (tps 129..1024): the rule's double-buffered triples in Q8
# against the ring of three in consecutive order and the other triple orders, one-block
# (pitch) and planar layouts, two passes (tools/order_ab.py). Usage: bash tools/mid_shard_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-mid}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for s in 10,4,1677722,182 12,4,1398102,191 12,4,5592406,47 8,4,8388608,42 10,4,6710887,45 8,4,2097152,170 16,4,2097152,96 10,4,4194304,64 8,4,4194304,85; do
  A+=(--shape "$s,-,pitch" --shape "$s,-,planar")
done
for pass in 1 2; do
  timeout -k 10 500 python3 -u tools/order_ab.py --rounds 3 --orders consecutive,q8,tri-q8,tri,tri-g2,tri-x32 \
    "${A[@]}" > "$O/ab$pass.jsonl" 2>&1 || exit $?
  echo "pass $pass ok"
done
