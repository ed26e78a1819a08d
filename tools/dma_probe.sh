# LDS-DMA ring (rs_apply.hpp Policy::DMA, A/B build): bit-exact through the every-order test
# on the A/B library, then against the rule and the triple forms on R 5..8 and R <= 4 shapes
# (tools/order_ab.py, planar layout). Usage: bash tools/dma_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-dma}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
# the A/B build is not pushed: built here on demand (build/ab/, tools/callfs_rs_ab.h)
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
export CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k every_offered > "$O/pytest_ab.log" 2>&1 || exit $?
echo "ab tests ok"
A=()
for s in 10,8,6710887,32 8,8,8388608,32 8,8,2097152,128 10,8,1677722,128 32,8,2097152,64 \
         16,8,1048576,256 10,4,1048576,256 10,4,6710887,45 8,8,131072,1024; do
  A+=(--shape "$s,-,planar")
done
timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 \
  --orders consecutive,g2,x32,tri,tri-g2,tri-x32,tri-q8,dma,dma-g2,dma-q8,dma-x32 "${A[@]}" \
  > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
