# A/B of the XCD-grouped tile orders (tile_order.hpp block_tile): the same shapes under
# CALLFS_RS_TILE_ORDER unset (the rule) / x8 / x32, alternated twice, one process each.
# Usage: bash tools/xcd_order_ab.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-xcd}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k every_offered_order > "$OUT/pytest_orders.log" 2>&1 \
  || { tail -30 "$OUT/pytest_orders.log"; exit 1; }
echo "pytest orders: $(tail -1 "$OUT/pytest_orders.log")"
SHAPES="--shape 10,4,6710887,64,-,split --shape 10,4,6710896,64,-,contig --shape 10,4,1048592,256,-,contig --shape 10,4,1048576,256 --shape 10,4,6710887,64,5,split"
for rep in 1 2; do
  for ord in rule x8 x32; do
    if [ "$ord" = rule ]; then unset CALLFS_RS_TILE_ORDER; else export CALLFS_RS_TILE_ORDER=$ord; fi
    timeout -k 10 300 python3 -u tools/ceiling_sweep.py $SHAPES > "$OUT/${ord}_$rep.jsonl" 2> "$OUT/${ord}_$rep.err" || exit $?
    echo "$ord $rep ok"
  done
done
unset CALLFS_RS_TILE_ORDER
# bit-exactness of the X8 / X32 instances (plain, Verify and realigning kernels) under the
# override: the misaligned / Split-layout / random-plan / tile-order tests
for ord in x8 x32; do
  CALLFS_RS_TILE_ORDER=$ord timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "misaligned or split or realign or random_plan or tile or tune or decode_rs10" > "$OUT/pytest_$ord.log" 2>&1 || { tail -20 "$OUT/pytest_$ord.log"; exit 1; }
  echo "pytest $ord: $(tail -1 "$OUT/pytest_$ord.log")"
done
