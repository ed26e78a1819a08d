# 6-bit triple lookups (Policy::WIX) against the rule's nibble kernel: bit-exact tests, the
# LDS lookup-rate probe, then interleaved A/B on R <= 4 shapes (tools/order_ab.py).
# Usage: bash tools/wix_ab.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-wix}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "wix or every_offered_order" > "$OUT/pytest_wix.log" 2>&1 || { tail -30 "$OUT/pytest_wix.log"; exit 1; }
tail -2 "$OUT/pytest_wix.log"
timeout -k 10 120 tools/lds_rate 2000 > "$OUT/lds_rate.txt" 2>&1 || exit $?
cat "$OUT/lds_rate.txt"
timeout -k 10 600 python3 -u tools/order_ab.py --orders wix,wix-g2,wix-x32 --rounds 4 \
  --shape 10,4,1048576,256 --shape 20,4,1048576,256 --shape 32,4,1048576,128 \
  --shape 16,4,1048576,256 --shape 12,4,1048576,256 --shape 4,2,1048576,512 \
  --shape 6,3,1048576,256 --shape 10,4,104864,2000 --shape 20,2,1048576,256 \
  > "$OUT/ab.jsonl" 2>&1 || { tail -20 "$OUT/ab.jsonl"; exit 1; }
cat "$OUT/ab.jsonl"
