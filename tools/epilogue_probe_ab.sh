# Epilogue probes for R = 4 launches (CALLFS_RS_PROBE=3: block barrier before a full tile's
# stores; 4: raised wave priority while storing) against production, alternated.
# Usage: bash tools/epilogue_probe_ab.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-probe}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R"
SH="--shape 10,4,1048576,256 --shape 10,4,1048576,256,0+1+2+3 --shape 16,4,1048576,128 --shape 10,4,6710887,64 --shape 20,4,1048576,128"
for i in 1 2; do
  for p in 0 3 4; do
    CALLFS_RS_PROBE=$p timeout -k 10 300 python3 -u tools/ceiling_sweep.py --rounds 3 --tune 1 --only prod,tuned $SH > "$OUT/p${p}_$i.jsonl" 2> "$OUT/p${p}_$i.err" || { tail -5 "$OUT/p${p}_$i.err"; exit 1; }
  done
done
echo ok
