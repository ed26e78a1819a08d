# Full GPU pass: gpu tests, default bench, rocprofv3 passes. Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-r01}"
cd "$R"; mkdir -p "gpurun_out/$TAG"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > "gpurun_out/$TAG/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 "gpurun_out/$TAG/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/$TAG/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 "gpurun_out/$TAG/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "gpurun_out/$TAG/bench.log" 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 "gpurun_out/$TAG/bench.log"; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh "$TAG"
