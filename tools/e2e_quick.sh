set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cpuab
make -s -C oracle -B
for rep in 1 2; do
ORC_GFNI_GENERIC=1 timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 8 > gpurun_out/cpuab/generic_$rep.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-seconds 8 > gpurun_out/cpuab/special_$rep.log 2>&1 || exit $?
done
echo ok
