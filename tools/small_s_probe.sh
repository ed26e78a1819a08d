# Small shards (1 MiB objects): throughput and memory-side read latency against the tiles
# in flight. The production dispatch (one tile per block) beside persistent grids of 1..4
# blocks per CU (tools/kbench KB_PERSIST), then per variant a PMC pass of the L2's memory
# read queue (latency = TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ, Little's law).
# Usage: bash tools/small_s_probe.sh <tag>; table: python tools/small_s_table.py <dir>
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-small_s}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
C="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_CYCLE_sum"
for sh in "10 4 104858 2925" "10 8 104858 2275" "20 4 52429 3413" "10 4 1677722 182"; do
  set -- $sh; k=$1; m=$2; S=$3; B=$4
  KB_PERSIST=1 KB_KEEP="persist" timeout -k 10 150 "$R/tools/kbench" $k $m $S $B 5 10 > "$OUT/time_${k}_${m}_$S.log" 2>&1 || exit $?
  for v in "prod dispatch" "persist 1" "persist 2" "persist 3" "persist 4"; do
    tag=$(echo "$v" | tr ' ' '_')
    KB_PERSIST=1 KB_ONLY="$v" timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${k}_${m}_${S}_$tag" -o pmc -- \
      "$R/tools/kbench" $k $m $S $B 1 3 > "$OUT/pmc_${k}_${m}_${S}_$tag.log" 2>&1
    rc=$?
    case $rc in 0) ;; 124|134|137|139) echo "pmc $v $k,$m,$S ended rc=$rc: stop"; exit $rc ;;
      *) echo "pmc $v $k,$m,$S failed rc=$rc"; tail -3 "$OUT/pmc_${k}_${m}_${S}_$tag.log" ;; esac
  done
  echo "shape $k,$m,$S done"
done
