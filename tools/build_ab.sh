# Same-box A/B of an earlier build against HEAD on the production dispatch
# (tools/kbench "prod dispatch", encode), processes alternated per shape.
# tools/ab/kbench_<old> is built from `git archive <commit> callfs_amd/csrc tools/kbench.hip`
# with the kbench recipe (tools/kbench.hip header): r02 = 9c5d705 (round 2's final build),
# r03 = bfd0c6f (round 3's final build).
# Usage: bash tools/build_ab.sh <tag> <old: r02|r03> [reps] ["k m S" ...]
#   no shapes: the profile sweep's 33 cells (tools/profile_sweep.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-build_ab}"; OLD="${2:-r02}"; REPS="${3:-3}"
shift 3; mkdir -p "$OUT"
: > "$OUT/summary.txt"
shapes=("$@")
if [ ${#shapes[@]} -eq 0 ]; then
  for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
    set -- $km
    for L in 1048576 16777216 67108864; do shapes+=("$1 $2 $(( (L + $1 - 1) / $1 ))"); done
  done
fi
for sh in "${shapes[@]}"; do
  set -- $sh; k=$1; m=$2; S=$3
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  for rep in $(seq 1 "$REPS"); do
    for v in "$OLD" head; do
      bin=tools/kbench; [ $v = "$OLD" ] && bin=tools/ab/kbench_$OLD
      log="$OUT/kb_${k}_${m}_${S}_${v}_$rep.log"
      KB_KEEP="@none@" timeout -k 10 120 $bin $k $m $S $B 5 10 > "$log" 2>&1 || exit $?
      echo "RS($k,$m) S=$S B=$B $v rep$rep $(grep 'prod dispatch' "$log" | awk '{print $(NF-1), $NF}')" | tee -a "$OUT/summary.txt"
    done
  done
done
