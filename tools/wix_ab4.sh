# WIX (6-bit lookups) vs Tri (same triple loads, nibble lookups) vs the nibble ring, encode
# shapes and launches with Verify rows (downloads, codec.go:59). Usage: bash tools/wix_ab4.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-wix4}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python3 -u tools/order_ab.py --orders consecutive,g2,x32,wix,wix-g2,wix-x32,tri,tri-g2,tri-x32 --rounds 4 \
  --shape 4,2,1048576,512 --shape 5,3,1048576,256 --shape 8,4,1048576,256 --shape 10,4,1048576,256 \
  --shape 8,8,1048576,256 --shape 6,6,1048576,256 --shape 10,8,1048576,256 \
  --shape 4,2,1048576,512,none --shape 4,2,1048576,512,1 --shape 6,3,1048576,256,2 \
  --shape 8,4,1048576,256,5 --shape 10,4,1048576,256,5 --shape 10,4,1048576,256,none \
  > "$OUT/ab.jsonl" 2>&1 || { tail -20 "$OUT/ab.jsonl"; exit 1; }
cat "$OUT/ab.jsonl"
