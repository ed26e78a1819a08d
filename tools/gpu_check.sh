# GPU-box check: gpu tests + short bench. Usage: bash tools/gpu_check.sh [pytest args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -q --maxfail=10 -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench1.log 2>&1; echo "bench rc=$?"
tail -2 gpurun_out/bench1.log
