# quick GPU check: pytest -m gpu (optionally -k filter) then bench. Usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-quick}"; mkdir -p "$OUT"
K=(); [ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --cpu-seconds 3 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-200
