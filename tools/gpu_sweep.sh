set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sweep
for cfg in "10 4 1048576 256" "10 4 6710887 64" "16 4 262144 1024" "16 4 4194304 64" "3 2 349526 1024" "10 1 1048576 256" "10 8 1048576 256" "4 2 1048576 512" "20 4 1048576 128" "32 8 1048576 64"; do
  timeout -k 10 120 tools/kbench $cfg 5 10 > "gpurun_out/sweep/kb_${cfg// /_}.log" 2>&1 || exit $?
done
echo kbench done
timeout -k 10 400 python3 tools/e2e_bench.py --threads 1 > gpurun_out/sweep/e2e_t1.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/e2e_bench.py --threads 8 --sizes 64K,1M,16M,64M > gpurun_out/sweep/e2e_t8.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/e2e_bench.py --k 10 --m 4 --erase 0,1,2,3 --sizes 10M,64M,1G --threads 1 --seconds 3 > gpurun_out/sweep/e2e_rs10.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/e2e_bench.py --k 3 --m 2 --erase 1 --sizes 1M --threads 1 --seconds 3 > gpurun_out/sweep/e2e_rs3.log 2>&1 || exit $?
echo e2e done
