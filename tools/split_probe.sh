# Split-layout (pitch = S) vs aligned layouts, production and ceilings. Usage: bash tools/split_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-split}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 3 \
  --shape 10,4,6710887,64,-,split --shape 10,4,6710896,64,-,contig --shape 10,4,6711040,64,-,contig \
  --shape 10,4,6710887,64 --shape 10,4,6710896,64,-,split --shape 10,4,1048577,256,-,split \
  --shape 10,4,1048576,256,-,contig --shape 10,4,1048592,256,-,contig --shape 10,4,1048577,256 \
  > "$OUT/split.jsonl" 2> "$OUT/split.err" || { tail -5 "$OUT/split.err"; exit 1; }
echo ok
