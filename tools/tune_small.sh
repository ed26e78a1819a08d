# rs_plan_tune vs the rule on 1 MiB objects (small shards, many stripes): encode plans.
# Usage: bash tools/tune_small.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tsmall}"; mkdir -p "$OUT"
for km in "10 4" "6 3" "10 8" "20 4" "4 2" "16 4"; do
  set -- $km; k=$1; m=$2
  S=$(( (1048576 + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) ))
  timeout -k 10 300 python3 tools/decode_sweep.py --tune 1 --patterns "enc;" --k $k --m $m --shard-bytes $S --stripes $B > "$OUT/rs${k}_${m}.jsonl" 2>&1 || exit $?
  grep '^{' "$OUT/rs${k}_${m}.jsonl" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print('RS($k,$m)', d['S'], d['stripes'], d['plan'], d['frac_8TBs'], d['tile_order'])"
done
