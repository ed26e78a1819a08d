# (round 2: compile-time-K variants measured 1-3 points slower than the runtime-K kernel
#  except RS(4,2)/RS(8,4) +1; RS(10,8) spilled. Removed; profiles/r02/kt_sweep/ keeps the logs.)
# Compile-time K (fully unrolled shard loop, counted waits) vs the runtime-K production
# kernel. Usage: bash tools/kt_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-kt}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_KT=1 KB_KEEP="kt |rt g2|nomath g2"
while read k m S B; do
  name="kbench_${k}_${m}_${S}_${B}"
  timeout -k 10 200 "$R/tools/kbench" $k $m $S $B 7 10 > "$OUT/$name.log" 2>&1 || exit $?
  grep -E "^(prod|kt|rt|nomath)|MISMATCH" "$OUT/$name.log" | sed "s/^/RS($k,$m) S=$S B=$B /"
done <<'LIST'
10 4 1048576 256
4 2 1048576 512
10 8 1048576 256
16 4 1048576 256
6 3 1048576 256
8 4 1048576 256
10 4 6710887 64
LIST
