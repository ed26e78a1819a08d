# Is the kernel's compute exposed? The production launch against its no-lookup form (same
# loads, stores, grid, order; A/B build) and the read / write ceilings, on R 5..8 and wide
# shapes and on the bench shape (tools/ceiling_sweep.py). Usage: bash tools/nolookup_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-nolookup}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
# the A/B build is not pushed: built here on demand (build/ab/, tools/callfs_rs_ab.h)
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
export CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so"
A=()
for s in 10,4,1048576,256 10,4,6710887,64 10,8,6710887,32 8,8,8388608,32 32,8,2097152,64 \
         16,8,1048576,256 10,16,1048576,128 20,16,1048576,96 32,16,1048576,64; do
  A+=(--shape "$s,-,planar")
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --rounds 2 "${A[@]}" > "$O/sweep.jsonl" 2>&1 || exit $?
echo "nolookup ok"
