# Round-end evidence in one call: GPU tests, smoke, bench line, rocprofv3 passes (gpu_round.sh),
# one pass of the planar rule sweep, and the write-pattern probe. Usage: bash tools/round_final.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-final}"; cd "$R"
bash tools/gpu_round.sh "$TAG" || exit $?
A=()
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,planar")
  done
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "gpurun_out/$TAG/rule_sweep.jsonl" 2>&1 || exit $?
echo "rule sweep ok"
timeout -k 10 300 tools/write_pattern 6 > "gpurun_out/$TAG/write_pattern_bs.csv" 2>&1 || exit $?
echo "write pattern ok"
# the double-buffered triples with 4 / 8 stripes interleaved (A/B build): bit-exact, then
# against the rule's tri-G2 on the bench shape and its neighbours
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so" timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py -k every_offered > "gpurun_out/$TAG/pytest_ab.log" 2>&1 || exit $?
echo "ab tests ok"
A=()
for s in 10,4,1048576,256 10,4,1048576,512 16,4,1048576,256 8,4,2097152,128 12,4,1398102,128 10,4,104858,1024 6,3,174763,2048; do
  A+=(--shape "$s,-,planar")
done
CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so" timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 \
  --orders tri-g2,tridb-g4,tridb-g8,tri-x32 "${A[@]}" > "gpurun_out/$TAG/tridb_g.jsonl" 2>&1 || exit $?
echo "tridb-g ok"
