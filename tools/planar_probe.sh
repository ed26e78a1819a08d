# The 256-B-pitch batch with every stripe's data and parity in one block ([b][n][pitch],
# 'pitch') against data and parity in two regions ([b][k][pitch] + [b][m][pitch],
# 'planar'), same shapes, rule and triple orders (tools/order_ab.py), two passes in
# alternated order; then the Split layout of an io.ReadAll body under the rule.
# Usage: bash tools/planar_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-planar}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
SH="10,4,1048576,256 10,4,104858,1024 12,4,87382,1024 10,8,104858,1024 20,4,52429,1024 4,2,262144,2048 6,3,174763,2048 8,4,2097152,128 4,2,16777216,32 10,4,6710887,64"
for pass in 1 2; do
  for L in pitch planar; do
    [ $pass = 2 ] && L=$([ $L = pitch ] && echo planar || echo pitch)
    A=(); for s in $SH; do A+=(--shape "$s,-,$L"); done
    timeout -k 10 400 python3 -u tools/order_ab.py --rounds 2 --orders tri-g2,tri-x32,tri-q8 "${A[@]}" \
      > "$O/${L}_$pass.jsonl" 2>&1 || exit $?
    echo "$L $pass ok"
  done
done
A=(); for s in 10,4,6710887,64 10,4,104858,1024 12,4,87382,1024 5,3,209716,1024 6,3,174763,2048 10,8,1048577,256; do
  A+=(--shape "$s,-,readall" --shape "$s,0+1+2,readall"); done
timeout -k 10 400 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 "${A[@]}" > "$O/readall_rule.jsonl" 2>&1 || exit $?
echo "readall ok"
timeout -k 10 300 python3 bench.py --shard-bytes 6710887 --stripes 256 --split-layout readall --steps 20 \
  --cpu-seconds 0 > "$O/bench_readall.log" 2>&1 || exit $?
echo "bench readall ok"
