# LDS-kernel tile orders over shard sizes (KB_ORD variants of tools/kbench).
# Usage: bash tools/order_sweep.sh <tag> "k m S B" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/$1"; shift; mkdir -p "$OUT"
for shape in "$@"; do
  set -- $shape
  KB_ORD=1 KB_KEEP="${KB_KEEP:-lds prod-policy|lds ord|read-only|write-only}" timeout -k 10 120 tools/kbench $1 $2 $3 $4 ${KB_ROUNDS:-7} 10 > "$OUT/kb_$1_$2_$3_$4.log" 2>&1 || exit $?
  echo "== $shape"; grep -v "^RS" "$OUT/kb_$1_$2_$3_$4.log" | awk '{print $1,$2,$3,$4,$NF}'
done
