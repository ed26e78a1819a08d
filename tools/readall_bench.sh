# configs[1]/[2] shape in the layouts upstream produces: bench.py at S = 6,710,887 with the
# io.ReadAll Split layout (decode into fresh buffers, as Reconstruct allocates them, and in
# place) and the planar layout; plus the bench shape. Usage: bash tools/readall_bench.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-readall}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
run() { timeout -k 10 300 python3 -u bench.py --steps 20 --cpu-seconds 0 --layout-ab 0 "$@"; }
run --shard-bytes 6710887 --split-layout readall > "$O/readall_fresh.log" 2>&1 || exit $?
run --shard-bytes 6710887 --split-layout readall --decode-into inplace > "$O/readall_inplace.log" 2>&1 || exit $?
run --shard-bytes 6710887 > "$O/planar_cfg12.log" 2>&1 || exit $?
run > "$O/planar_bench.log" 2>&1 || exit $?
echo "benches ok"
