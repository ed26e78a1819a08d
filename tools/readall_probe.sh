# Split layout of an io.ReadAll body (parity in AllocAligned buffers) beside the
# all-contiguous Split layout: production rule, tuned, ceilings; then every kernel form in
# the readall layout; then the driver's line in both layouts.
# Usage: bash tools/readall_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-readall}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
SH=""
for s in 10,4,6710887,64 4,2,1048577,512 6,3,1048577,256 10,8,1048577,256 12,4,5592406,64 \
         5,3,209716,1024 10,4,104858,1024; do
  SH="$SH --shape $s,-,split --shape $s,-,readall"
done
timeout -k 10 400 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 $SH > "$O/sweep.jsonl" 2>&1 || exit $?
echo "sweep ok"
timeout -k 10 300 python3 -u tools/order_ab.py --rounds 3 \
  --orders realign,realign-x8,realign-x32,realign-tri-x32,consecutive,g2,x8,x32,q8 \
  --shape 10,4,6710887,64,-,readall --shape 6,3,1048577,256,-,readall \
  --shape 4,2,1048577,512,-,readall --shape 10,8,1048577,256,-,readall > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
for L in readall split; do
  timeout -k 10 300 python3 bench.py --shard-bytes 6710887 --stripes 256 --split-layout $L --steps 20 \
    --cpu-seconds 0 > "$O/bench_$L.log" 2>&1 || exit $?
  echo "bench $L ok"; tail -c 600 "$O/bench_$L.log"
done
