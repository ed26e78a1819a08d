# Split layout of an io.ReadAll body (parity in AllocAligned buffers) beside the
# all-contiguous Split layout: production rule, tuned, ceilings; then every kernel form in
# the readall layout (the 64-vector realigning form REALIGN 5, the ring-of-three and
# triple realigning forms, the plain kernel's unaligned accesses); then the driver's line
# in both layouts. Usage: bash tools/readall_probe.sh <tag> [skip-sweep]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-readall}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
SHAPES="10,4,6710887,64 4,2,1048577,512 6,3,1048577,256 10,8,1048577,256 12,4,5592406,64 5,3,209716,1024 10,4,104858,1024"
if [ -z "$2" ]; then
  SH=""
  for s in $SHAPES; do SH="$SH --shape $s,-,split --shape $s,-,readall"; done
  timeout -k 10 400 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 $SH > "$O/sweep.jsonl" 2>&1 || exit $?
  echo "sweep ok"
fi
SH=""
for s in $SHAPES; do SH="$SH --shape $s,-,readall"; done
timeout -k 10 400 python3 -u tools/order_ab.py --rounds 3 \
  --orders realign-x32,realign64-x32,realign64,realign64-x8,realign-tri-x32,tri-x32,tri-g2,x32 \
  $SH > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
for L in readall split; do
  timeout -k 10 300 python3 bench.py --shard-bytes 6710887 --stripes 256 --split-layout $L --steps 20 \
    --cpu-seconds 0 > "$O/bench_$L.log" 2>&1 || exit $?
  echo "bench $L ok"; tail -c 300 "$O/bench_$L.log"
done
