# Cells where round 4's rule ran below round 3's build on the same box (profiles/r04/r03_ab):
# the round-3 build, HEAD, HEAD without the double-buffered form (CALLFS_RS_TRIDB=0) and
# HEAD without triples (CALLFS_RS_WIX=0), processes alternated, production dispatch.
# Usage: bash tools/regress_probe.sh <tag> ["k m S" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-regress}"; shift; mkdir -p "$OUT"; : > "$OUT/summary.txt"
shapes=("$@")
[ ${#shapes[@]} -eq 0 ] && shapes=("20 4 838861" "20 4 3355444" "8 4 8388608" "10 8 6710887" "20 4 1048576")
for sh in "${shapes[@]}"; do
  set -- $sh; k=$1; m=$2; S=$3
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  for rep in 1 2; do
    for v in r03 head notridb nowix; do
      bin=tools/kbench; envs=""
      case $v in r03) bin=tools/ab/kbench_r03;; notridb) envs="CALLFS_RS_TRIDB=0";; nowix) envs="CALLFS_RS_WIX=0";; esac
      log="$OUT/kb_${k}_${m}_${S}_${v}_$rep.log"
      env $envs KB_KEEP="@none@" timeout -k 10 120 $bin $k $m $S $B 5 10 > "$log" 2>&1 || exit $?
      echo "RS($k,$m) S=$S B=$B $v rep$rep $(grep 'prod dispatch' "$log" | awk '{print $(NF-1), $NF}')" | tee -a "$OUT/summary.txt"
    done
  done
done
