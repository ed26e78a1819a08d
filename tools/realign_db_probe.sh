# The realigning kernel (contiguous Split layout, misaligned outputs) with its aligned loads
# double-buffered in triples (REALIGN 2 + WIX 3, orders realign-tri*: R <= 4, K >= 6)
# against the ring of three (realign*), encode and decodes (tools/order_ab.py).
# Usage: bash tools/realign_db_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-rdb}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for s in 10,4,6710887,64 6,3,1048577,256 12,4,5592406,64 10,4,104858,1024 12,4,87382,1024 16,4,262145,256 8,4,1048577,256 20,4,838861,128; do
  A+=(--shape "$s,-,split")
done
A+=(--shape 10,4,6710887,64,0+1+2+3,split --shape 10,4,6710887,64,5,split --shape 10,4,104858,1024,0+1+2+3,split)
timeout -k 10 500 python3 -u tools/order_ab.py --rounds 3 --orders realign-x32,realign-x8,realign-tri-x32,realign-tri-x8,realign-tri \
  "${A[@]}" > "$O/ab.jsonl" 2>&1 || exit $?
echo "ab ok"
