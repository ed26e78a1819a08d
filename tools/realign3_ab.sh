# REALIGN 3 (edge vectors through LDS, 64 per wave) vs REALIGN 2: the misaligned-layout GPU
# tests with it forced, then alternated sweeps. Usage: bash tools/realign3_ab.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-ra3}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
CALLFS_RS_REALIGN=3 timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "realign or misaligned or split or random_plans or tune" > "$OUT/pytest_ra3.log" 2>&1 || { tail -30 "$OUT/pytest_ra3.log"; exit 1; }
tail -1 "$OUT/pytest_ra3.log"
SH="--shape 10,4,6710887,64,-,split --shape 10,4,1048577,256,-,split --shape 10,8,1048577,256,-,split --shape 4,2,1048577,512,-,split --shape 6,3,1048577,256,-,split --shape 10,4,6710896,64,-,contig"
for i in 1 2; do
  for v in 2 3; do
    CALLFS_RS_REALIGN=$v timeout -k 10 300 python3 -u tools/ceiling_sweep.py --rounds 3 --only prod $SH > "$OUT/ra${v}_$i.jsonl" 2> "$OUT/ra${v}_$i.err" || exit 1
  done
done
echo ok
