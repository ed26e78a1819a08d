# Runs one gpurun call; repeats it only while gpurun reports an infrastructure event
# (status "transient" or exit 3: no box, nothing charged, nothing ran), at most 20 times.
# A command that ran and failed is never repeated.
# Usage: bash tools/gpurun_retry.sh <timeout_s> <log> '<command>'
t=$1; log=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1; rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = 3 ] || { [ "$st" = transient ] && grep -q "retry" "$log"; }; then
    w=$(grep -o "retry in [0-9]*s" "$log" | tail -1 | tr -dc 0-9); w=${w:-90}; w=$((w + 60))
    echo "attempt $i: infrastructure ($rc/$st), retrying in $w s" >> "$log.retries"; sleep "$w"; continue
  fi
  exit $rc
done
exit $rc
