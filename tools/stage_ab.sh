# REALIGN 4 (parity stores staged through LDS, written from 128-B boundaries) vs REALIGN 2:
# forced-order parity tests, then tools/order_ab.py on Split-layout shapes, two processes.
# Usage: bash tools/stage_ab.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-stage}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "every_offered_order or misaligned or split or tune" \
  > "$OUT/pytest_orders.log" 2>&1 || { tail -30 "$OUT/pytest_orders.log"; exit 1; }
echo "pytest: $(tail -1 "$OUT/pytest_orders.log")"
ORD="realign,realign-x32,stage,stage-x8,stage-x32,consecutive"
SHAPES="--shape 10,4,6710887,64,-,split --shape 10,4,1048577,256,-,split --shape 10,4,6710887,64,5,split --shape 10,4,6710887,64,0+1+2+3,split --shape 10,8,1048577,256,-,split --shape 4,2,1048577,512,-,split --shape 6,3,1048577,256,-,split --shape 12,4,5592406,64,-,split"
for rep in 1 2; do
  timeout -k 10 400 python3 -u tools/order_ab.py --orders "$ORD" $SHAPES > "$OUT/ab_$rep.jsonl" 2> "$OUT/ab_$rep.err" || exit $?
  echo "ab $rep ok"
done
cat "$OUT"/ab_*.jsonl
