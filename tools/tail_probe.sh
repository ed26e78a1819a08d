# Cost of the ragged tail (S % 16) at 1 MiB-object shard sizes: the production dispatch
# at S = ceil(L/k) against the nearest multiple of 16 below it, same batch (tools/kbench).
# Usage: bash tools/tail_probe.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tail_probe}"; mkdir -p "$OUT"; : > "$OUT/summary.txt"
for sh in "10 4 104858" "10 8 104858" "20 4 52429" "6 3 174763" "12 4 87382" "5 3 209716"; do
  set -- $sh; k=$1; m=$2; S=$3; S16=$(( S / 16 * 16 ))
  B=$(( (4 << 30) / (S * (k + m)) ))
  for rep in 1 2; do
    for s in $S $S16; do
      KB_KEEP="@none@" timeout -k 10 120 tools/kbench $k $m $s $B 5 10 > "$OUT/kb_${k}_${m}_${s}_$rep.log" 2>&1 || exit $?
      echo "RS($k,$m) S=$s B=$B rep$rep $(grep 'prod dispatch' "$OUT/kb_${k}_${m}_${s}_$rep.log" | awk '{print $(NF-1), $NF}')" | tee -a "$OUT/summary.txt"
    done
  done
done
