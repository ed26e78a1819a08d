# configs[1]/[2] shape (RS(10,4), S = 6,710,887, planar) against neighbouring shard sizes:
# every tile order and kernel form the plan offers (tools/order_ab.py), to tell a shard-size
# effect from an order effect. Usage: bash tools/cfg12_orders.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-cfg12o}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
ORD=consecutive,g2,q8,q16,x8,x32,tri,tri-g2,tri-q8,tri-q16,tri-x8,tri-x32
A=()
for s in 10,4,6710887,45,- 10,4,6710887,45,0+1+2+3 10,4,6710880,45,- 10,4,8388608,36,- \
         10,4,4194304,73,- 10,4,2097152,146,- 10,4,1048576,292,- 10,4,6710887,256,-; do
  A+=(--shape "$s,planar")
done
timeout -k 10 900 python3 -u tools/order_ab.py --rounds 3 --orders "$ORD" "${A[@]}" \
  > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
