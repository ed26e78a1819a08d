# One-erasure decodes (written + Verify rows, R <= 4): the ring of three with early compare
# loads (the rule) against the triple loop with early compare loads (Policy::WIX 2 + VPF),
# interleaved in one process (tools/order_ab.py). Usage: bash tools/tri_verify_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tri_verify_ab}"; mkdir -p "$OUT"
timeout -k 10 600 python -u tools/order_ab.py --rounds 4 --orders consecutive,g2,x32,tri,tri-g2,tri-x32,tri-q8 \
  --shape 10,4,1048576,256,5 --shape 10,4,1048576,256,13 --shape 10,4,1048576,256,0 \
  --shape 6,3,1048576,455,2 --shape 8,4,1048576,341,5 --shape 4,2,1048576,682,1 \
  --shape 4,2,4194304,170,0 --shape 10,4,6710887,45,5 --shape 16,4,1048576,204,3 \
  --shape 12,4,1048576,256,7 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || exit $?
