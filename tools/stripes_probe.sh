# Does the best form at long shards depend on the batch size? RS(10,4) at 6.7 MB and 8 MiB
# shards with 45..256 stripes, the ring (consecutive) against the triple forms (tools/order_ab.py).
# Usage: bash tools/stripes_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-stripes}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for s in 10,4,6710887,45 10,4,6710887,128 10,4,6710887,256 10,4,8388608,36 10,4,8388608,128 \
         10,4,8388608,200 12,4,5592406,54 12,4,5592406,256; do
  A+=(--shape "$s,-,planar")
done
timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 --orders consecutive,x32,tri-q8,tri-x32 "${A[@]}" \
  > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
