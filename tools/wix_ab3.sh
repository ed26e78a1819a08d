# WIX vs the nibble kernel: K = 4..12, R = 1..4, 1 MiB shards and 1 MiB objects. Usage: bash tools/wix_ab3.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-wix3}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python3 -u tools/order_ab.py --orders consecutive,g2,g8,x32,wix,wix-g2,wix-g8,wix-x32 --rounds 4 \
  --shape 4,2,262144,2048 --shape 4,1,1048576,512 --shape 4,4,1048576,384 --shape 5,2,1048576,512 \
  --shape 7,3,1048576,256 --shape 9,4,1048576,256 --shape 6,2,1048576,384 --shape 8,2,1048576,384 \
  --shape 10,2,1048576,256 --shape 12,3,1048576,256 --shape 8,4,131072,2048 --shape 5,3,209716,2048 \
  > "$OUT/ab.jsonl" 2>&1 || { tail -20 "$OUT/ab.jsonl"; exit 1; }
cat "$OUT/ab.jsonl"
