# Launch-slice size (CALLFS_RS_MAX_TILES_PER_LAUNCH, rs_kernels.hip slice_tiles) on the
# configs[1] shape (RS(10,4), S = 6,710,887, planar, 256 stripes = 24 GB per launch) and on
# the bench shape, rule and tuned plus the read / write ceilings; one process per setting.
# Usage: bash tools/slice_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-slice}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
for T in 0 4096 8192 16384 65536 1000000000; do
  if [ $T = 0 ]; then unset CALLFS_RS_MAX_TILES_PER_LAUNCH; else export CALLFS_RS_MAX_TILES_PER_LAUNCH=$T; fi
  timeout -k 10 300 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned,read,write \
    --shape 10,4,6710887,256,-,planar --shape 10,4,6710887,256,0+1+2+3,planar \
    --shape 10,4,1048576,256,-,planar > "$O/slice_$T.jsonl" 2>&1 || exit $?
  echo "slice $T ok"
done
