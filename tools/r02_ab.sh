# Same-box A/B of the round-2 build (9c5d705) against HEAD on the production dispatch
# (tools/kbench "prod dispatch", encode), processes alternated per shape.
# tools/ab/kbench_r02 is built from `git archive 9c5d705 callfs_amd/csrc tools/kbench.hip`
# with the kbench recipe (tools/kbench.hip header).
# Usage: bash tools/r02_ab.sh <tag> ["k m S" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-r02_ab}"; shift; mkdir -p "$OUT"
: > "$OUT/summary.txt"
shapes=("$@")
[ ${#shapes[@]} -eq 0 ] && shapes=("4 2 4194304" "4 2 16777216" "6 3 2796203" "6 3 11184811" "8 8 8388608" "4 2 262144" "10 4 1048576")
for sh in "${shapes[@]}"; do
  set -- $sh; k=$1; m=$2; S=$3
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  for rep in 1 2 3; do
    for v in r02 head; do
      bin=tools/kbench; [ $v = r02 ] && bin=tools/ab/kbench_r02
      log="$OUT/kb_${k}_${m}_${S}_${v}_$rep.log"
      KB_KEEP="@none@" timeout -k 10 120 $bin $k $m $S $B 5 10 > "$log" 2>&1 || exit $?
      echo "RS($k,$m) S=$S B=$B $v rep$rep $(grep 'prod dispatch' "$log" | awk '{print $(NF-1), $NF}')" | tee -a "$OUT/summary.txt"
    done
  done
done
