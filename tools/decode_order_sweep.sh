# Decode per erasure pattern under each forced LDS tile order (CALLFS_RS_TILE_ORDER is
# read once per process: one process per order), bench shape and 64 MiB-object shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG="${1:-dord}"; OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
for ord in rule consecutive g8 g2 q8 q16; do
  for shape in "--shard-bytes 1048576 --stripes 256" "--shard-bytes 6710887 --stripes 256"; do
    tagS=$(echo $shape | awk '{print $2}')
    if [ $ord = rule ]; then unset CALLFS_RS_TILE_ORDER; else export CALLFS_RS_TILE_ORDER=$ord; fi
    timeout -k 10 300 python3 tools/decode_sweep.py $shape > "$OUT/${ord}_${tagS}.jsonl" 2>&1 || exit $?
    python3 - "$OUT/${ord}_${tagS}.jsonl" "$ord" "$tagS" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
print(sys.argv[2], sys.argv[3], " ".join(f"{r['plan'].replace('decode erase ','')}:{r['frac_8TBs']*100:.1f}" for r in rows))
PY
  done
done
