# Misaligned shards (upstream Split layout, pitch = S odd): production dispatch against
# aligned loads + register realignment (KB_REALIGN), and which side pays (KB_OUT_SEP:
# outputs moved to aligned rows; KB_IN_SEP: inputs moved). Usage: bash tools/realign_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-realign}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_REALIGN=1 KB_KEEP="realign|nomath g2"
while read k m S B sep; do
  name="kbench_${k}_${m}_${S}_${B}_${sep}"
  case $sep in out) export KB_OUT_SEP=1; unset KB_IN_SEP;; in) export KB_IN_SEP=1; unset KB_OUT_SEP;;
    *) unset KB_OUT_SEP KB_IN_SEP;; esac
  timeout -k 10 200 "$R/tools/kbench" $k $m $S $B 5 8 1 > "$OUT/$name.log" 2>&1 || exit $?
  grep -E "^(prod|realign|nomath)|MISMATCH" "$OUT/$name.log" | sed "s/^/RS($k,$m) S=$S B=$B sep=$sep /"
done <<'LIST'
10 4 1048577 256 none
10 4 1048577 256 out
10 4 1048577 256 in
10 4 6710887 64 none
10 4 6710887 64 out
16 4 262145 256 none
16 4 262145 256 out
4 2 1048577 512 none
10 8 1048577 256 none
10 4 1048576 256 none
LIST
