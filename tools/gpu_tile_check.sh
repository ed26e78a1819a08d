# tile-order dispatch check: GPU tests, then kbench prod dispatch vs consecutive per shape, then bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tile}"; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for shape in "10 4 1048576 256" "16 4 1048576 256" "10 4 524288 512" "10 4 16777216 32" "16 4 16777216 16" "10 4 25165824 16" "10 4 67108864 8" "10 4 6710887 64" "10 4 13421824 32"; do
  set -- $shape
  KB_ORD=1 KB_KEEP="lds prod-policy" timeout -k 10 120 tools/kbench $1 $2 $3 $4 9 10 > "$OUT/kb_$1_$2_$3_$4.log" 2>&1 || exit $?
  echo "== $shape $(grep -h 'prod dispatch\|prod-policy' "$OUT/kb_$1_$2_$3_$4.log" | awk '{print $1,$2,$NF}' | tr '\n' ' ')"
done
timeout -k 10 300 python3 bench.py > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-400
