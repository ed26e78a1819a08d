# production dispatch vs consecutive tiles per shape (tools/kbench). Usage: bash tools/dispatch_check.sh <tag> "k m S B" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/$1"; shift; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "tile_orders or random_plans or plan_" > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for shape in "$@"; do
  set -- $shape
  KB_ORD=1 KB_KEEP="lds ord consec|lds ord g2|lds ord q16" timeout -k 10 120 tools/kbench $1 $2 $3 $4 9 10 > "$OUT/kb_$1_$2_$3_$4.log" 2>&1 || exit $?
  echo "== $shape $(grep -h 'prod dispatch\|lds ord' "$OUT/kb_$1_$2_$3_$4.log" | awk '{print $1,$2,$3,$NF}' | tr '\n' ' ')"
done
