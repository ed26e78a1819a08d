# GPU test suite only. Usage: bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-t}"; mkdir -p "$R/gpurun_out/$TAG"; cd "$R"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread "${K[@]}" > "gpurun_out/$TAG/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 "gpurun_out/$TAG/pytest_gpu.log"; exit $rc
