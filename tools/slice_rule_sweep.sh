# Launch-slice size vs grid size and shape (tools/kbench KB_SLICE: the production
# dispatch with slices of 1/2(rule)/4/8 GiB of traffic or none). Usage: bash tools/slice_rule_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-slice}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_SLICE=1 KB_KEEP="prod slice"
while read k m S B; do
  timeout -k 10 240 "$R/tools/kbench" $k $m $S $B 5 6 > "$OUT/kbench_${k}_${m}_${S}_${B}.log" 2>&1 || exit $?
  grep -E "^prod" "$OUT/kbench_${k}_${m}_${S}_${B}.log" | sed "s/^/RS($k,$m) S=$S B=$B /"
done <<'LIST'
10 4 1048576 256
10 4 1048576 512
10 4 1048576 1024
10 4 6710887 256
10 8 1048576 256
10 8 1048576 1024
10 12 1048576 256
10 16 1048576 256
20 16 1048576 256
32 16 1048576 256
32 8 1048576 256
20 4 1048576 256
4 2 1048576 2048
16 4 4194304 64
LIST
