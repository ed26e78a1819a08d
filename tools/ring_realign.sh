# Branch-free prefetch rings and aligned-load realignment A/B. Usage: bash tools/ring_realign.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-ring}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
# (round 2 measured RING 2/3 -- clamped prefetch index, static unrolled slots -- 1-12 points
# slower than RING 0 and removed them; this script now reruns only the realign A/B)
export KB_REALIGN=1 KB_KEEP="realign|nomath g2"
while read k m S B pal; do
  name="kbench_${k}_${m}_${S}_${B}_${pal}"
  timeout -k 10 200 "$R/tools/kbench" $k $m $S $B 5 8 $pal > "$OUT/$name.log" 2>&1 || exit $?
  grep -E "^(prod|ring|realign|nomath)|MISMATCH" "$OUT/$name.log" | sed "s/^/RS($k,$m) S=$S B=$B pal=$pal /"
done <<'LIST'
10 4 1048576 256 256
10 4 1048577 256 1
10 4 6710887 64 1
4 2 1048576 512 256
10 8 1048576 256 256
20 4 1048576 256 256
16 4 262145 256 1
LIST
