# A/B of the 8-byte-per-lane wide kernel (CALLFS_RS_WIDE_HALF=1) against production for
# R 9..16 groups: GPU tests with it on, then alternated ceiling sweeps. Usage: bash tools/wide_half_ab.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-half}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
CALLFS_RS_WIDE_HALF=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_half.log" 2>&1 || { tail -20 "$OUT/pytest_half.log"; exit 1; }
tail -1 "$OUT/pytest_half.log"
SH="--shape 10,12,1048576,256 --shape 10,16,1048576,256 --shape 20,16,1048576,128 --shape 32,16,1048576,64 --shape 16,13,1048576,128 --shape 10,16,4194304,64"
for i in 1 2; do
  for h in 0 1; do
    CALLFS_RS_WIDE_HALF=$h timeout -k 10 300 python3 -u tools/ceiling_sweep.py --rounds 3 --only prod,nolookup $SH > "$OUT/half${h}_$i.jsonl" 2> "$OUT/half${h}_$i.err" || exit 1
  done
done
echo ok
