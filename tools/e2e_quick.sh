set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ua
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
KB_BYTES=1 KB_KEEP="byte-kernel" timeout -k 10 120 tools/kbench 10 4 1048577 256 5 10 1 > gpurun_out/ua/rs10_4.log 2>&1 || exit $?
KB_BYTES=1 KB_KEEP="byte-kernel" timeout -k 10 120 tools/kbench 10 4 6710887 64 5 10 1 > gpurun_out/ua/rs10_4_64m.log 2>&1 || exit $?
KB_BYTES=1 KB_KEEP="byte-kernel" timeout -k 10 120 tools/kbench 3 2 349526 1024 5 10 1 > gpurun_out/ua/rs3_2.log 2>&1 || exit $?
KB_BYTES=1 KB_KEEP="byte-kernel" timeout -k 10 120 tools/kbench 16 4 262145 256 5 10 1 > gpurun_out/ua/rs16_4.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/sha_bench.py > gpurun_out/ua/sha.json 2>&1 || exit $?
echo ok
