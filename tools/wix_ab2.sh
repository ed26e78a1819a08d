# WIX vs the nibble kernel in the same tile orders, few-input R <= 4 shapes. Usage: bash tools/wix_ab2.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-wix2}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python3 -u tools/order_ab.py --orders consecutive,g2,x32,wix,wix-g2,wix-x32 --rounds 5 \
  --shape 4,2,1048576,512 --shape 6,3,1048576,256 --shape 8,4,1048576,256 --shape 10,4,1048576,256 \
  --shape 12,4,1048576,256 --shape 4,2,4194304,128 --shape 10,4,1677722,180 --shape 5,3,1048576,256 \
  > "$OUT/ab.jsonl" 2>&1 || { tail -20 "$OUT/ab.jsonl"; exit 1; }
cat "$OUT/ab.jsonl"
