set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/zc gpurun_out/e2e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
O=gpurun_out/e2e/zerocopy.jsonl; rm -f $O
for pin in 0 1; do
  if [ $pin = 1 ]; then export CALLFS_E2E_PINNED=1; else unset CALLFS_E2E_PINNED; fi
  for L in 4096 65536 1048576 16777216 67108864; do timeout -k 10 60 tools/e2e_native 16 4 $L 1 1.0 0,5,16,19 >> $O || exit 1; done
  for L in 10485760 67108864 1073741824; do timeout -k 10 60 tools/e2e_native 10 4 $L 1 1.5 0,1,2,3 >> $O || exit 1; done
  CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 10 4 67108864 1 1.5 0,1,2,3 >> $O || exit 1
  timeout -k 10 60 tools/e2e_native 10 4 67108864 8 1.5 0,1,2,3 >> $O || exit 1
  timeout -k 10 60 tools/e2e_native 16 4 1048576 8 1.0 0,5,16,19 >> $O || exit 1
  timeout -k 10 60 tools/e2e_native 10 4 67108864 1 1.5 >> $O || exit 1
done
echo ok
