# The driver's bench line on this build, a wide-profile line (RS(20,16), 16 erasures: the
# bit-sliced kernels), and the A/B build's offered-order parity cases (the LDS-DMA ring with
# K below its depth). Usage: bash tools/bench_r06.sh <tag>
set -o pipefail
T=${1:-bench}; O=gpurun_out/r06/$T; mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2> $O/bench.err || exit $?
echo "bench ok"; tail -c 600 $O/bench.log
timeout -k 10 300 python3 -u bench.py --k 20 --m 16 --erase 0,1,2,3,4,5,6,7,20,21,22,23,24,25,26,27 \
  --layout-ab 0 --cpu-seconds 3 > $O/bench_rs20_16.log 2> $O/bench_rs20_16.err || exit $?
echo "wide bench ok"
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null 2> $O/build_ab.err || exit $?
CALLFS_RS_LIB=$PWD/build/ab/libcallfs_rs_ab.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py -k every_offered > $O/pytest_ab.log 2>&1 || exit $?
echo "ab tests ok"; tail -2 $O/pytest_ab.log
