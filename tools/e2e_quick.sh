set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ord3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
export KB_KEEP="lds prod-policy"
for cfg in "10 4 262144 1024" "10 4 1048576 256" "16 4 4194304 64" "10 4 6710887 128" "10 4 16777216 32" "16 4 65536 4096"; do
  timeout -k 10 120 tools/kbench $cfg 7 10 > "gpurun_out/ord3/kb_${cfg// /_}.log" 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --cpu-seconds 0 > gpurun_out/ord3/bench.log 2>&1 || exit $?
echo ok
