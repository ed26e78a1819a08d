# Cost of the ragged tail (S % 16) at small shards: kbench production dispatch at S with
# and without a tail. Usage: bash tools/tail_cost_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-tailcost}"; mkdir -p "$OUT"
export KB_KEEP="__none__"
for i in 1 2; do
for cfg in "10 8 104858 2275" "10 8 104848 2275" "20 4 52429 3413" "20 4 52432 3413" "10 4 104858 2925" "10 4 104864 2925" "3 2 349526 2457" "3 4 349526 1755"; do
  set -- $cfg
  timeout -k 10 120 "$R/tools/kbench" $1 $2 $3 $4 5 10 > "$OUT/kb_$1_$2_$3_$i.log" 2>&1 || exit $?
  echo "RS($1,$2) S=$3 run $i: $(grep '^prod dispatch' "$OUT/kb_$1_$2_$3_$i.log" | awk '{print $NF}')"
done
done
