# Ragged-tail placement A/B (rs_kernels.hip tail_mode): CALLFS_RS_TAIL_LAST_TPS=0 puts every
# tail in wave 0 of the stripe's first tile, the default (32) in the idle last wave of the
# last tile for stripes of <= 32 tiles, 1000000 in the last tile at every size; processes
# alternated, production dispatch (tools/kbench), plus S rounded down to 16 (no tail).
# Usage: bash tools/tail_ab.sh <tag> ["k m S" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tail_ab}"; shift; mkdir -p "$OUT"; : > "$OUT/summary.txt"
shapes=("$@")
[ ${#shapes[@]} -eq 0 ] && shapes=("20 4 52429" "10 8 104858" "12 4 87382" "6 3 174763" "3 2 349526"
  "20 4 838861" "10 4 1677722" "20 4 3355444" "10 4 6710887" "12 4 5592406" "6 3 11184811")
for sh in "${shapes[@]}"; do
  set -- $sh; k=$1; m=$2; S=$3
  B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
  for rep in 1 2; do
    for v in first t32 last flat; do
      s=$S; lim=""
      case $v in first) lim=0;; t32) lim=32;; last) lim=1000000;; flat) s=$(( S / 16 * 16 )); lim=32;; esac
      log="$OUT/kb_${k}_${m}_${S}_${v}_$rep.log"
      CALLFS_RS_TAIL_LAST_TPS=$lim KB_KEEP="@none@" timeout -k 10 120 tools/kbench $k $m $s $B 5 10 > "$log" 2>&1 || exit $?
      echo "RS($k,$m) S=$S B=$B $v rep$rep $(grep 'prod dispatch' "$log" | awk '{print $(NF-1), $NF}')" | tee -a "$OUT/summary.txt"
    done
  done
done
