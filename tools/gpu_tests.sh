# GPU test suite only. Usage: bash tools/gpu_tests.sh <tag> [pytest -k expr] [test path]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-t}"; mkdir -p "$R/gpurun_out/$TAG"; cd "$R"
K=()
[ -n "$2" ] && K=(-k "$2")
P="${3:-tests}"
timeout -k 10 900 python3 -u -m pytest "$P" -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread --durations 15 "${K[@]}" > "gpurun_out/$TAG/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 "gpurun_out/$TAG/pytest_gpu.log"; exit $rc
