# Triple-load rule check: GPU tests, smoke, bench, then the rule against nibble / WIX orders.
# Usage: bash tools/tri_check.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-tri}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
bash tools/gpu_tests.sh "$TAG" || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-1200
timeout -k 10 600 python3 -u tools/order_ab.py --orders consecutive,g2,x32,wix-g2,tri,tri-g2,tri-x32 --rounds 4 \
  --shape 4,2,1048576,512 --shape 4,2,262144,2048 --shape 10,4,1048576,256 --shape 10,4,1048576,256,0+1+2+3 \
  --shape 8,8,1048576,256 --shape 10,8,1048576,256 --shape 4,2,1048576,512,none --shape 6,3,174763,2048 \
  --shape 12,4,1048576,256 --shape 16,4,1048576,256 > "$OUT/ab.jsonl" 2>&1 || { tail -20 "$OUT/ab.jsonl"; exit 1; }
cat "$OUT/ab.jsonl"
