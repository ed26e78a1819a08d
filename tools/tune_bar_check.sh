# Tuner bar A/B (CALLFS_RS_TUNE_BAR 1 vs 0.5 %) on the bench shape and 1 MiB-object shapes,
# alternated, two rounds. Usage: bash tools/tune_bar_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tunebar}"; mkdir -p "$OUT"
j() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], round(d["roofline"]["frac"],4), round(d["roofline_decode"]["frac"],4), d["config"]["tile_order"])'; }
for i in 1 2; do
for cfg in "10 4 1048576 256 0,1,2,3" "4 2 262144 2048 0,1" "10 4 104858 2925 0,1,2,3" "16 4 65536 3413 0,1,2,3" "20 4 52429 3413 0,1,2,3"; do
  set -- $cfg
  for bar in 1 0.5; do
    CALLFS_RS_TUNE_BAR=$bar timeout -k 10 200 python3 bench.py --k $1 --m $2 --shard-bytes $3 --stripes $4 --erase $5 --steps 20 --warmup 5 --cpu-seconds 0 --ceiling 0 > "$OUT/rs$1_$2_$3_bar${bar}_$i.log" 2>&1 || exit $?
    echo "RS($1,$2) S=$3 bar $bar run $i: $(j $OUT/rs$1_$2_$3_bar${bar}_$i.log)"
  done
done
done
