# GPU tests (all), then an optional extra script. Usage: bash tools/gpu_tests_and.sh <tag> [script args...]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-t}"; shift
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
if [ $# -gt 0 ]; then bash "$@" || exit $?; fi
