set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ring2
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
export KB_KEEP="lds RT"
for cfg in "10 9 1048576 128" "10 12 1048576 128" "10 16 1048576 128" "20 16 1048576 64" "32 16 1048576 64" "4 13 1048576 128" "10 4 1048576 256"; do
  timeout -k 10 120 tools/kbench $cfg 5 10 > "gpurun_out/ring2/kb_${cfg// /_}.log" 2>&1 || exit $?
done
echo ok
