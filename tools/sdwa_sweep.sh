# LDS table address formation: v_or_b32_sdwa (byte select + OR) against v_perm_b32, same
# process, across narrow, wide and many-input shapes; plus the VALU issue rates.
# Usage: bash tools/sdwa_sweep.sh <tag> ["k,m k,m ..."]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-sdwa}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 60 "$R/tools/valu_rates" > "$OUT/valu_rates.log" 2>&1 || exit $?
cat "$OUT/valu_rates.log"
export KB_SDWA=1 KB_KEEP="sdwa|perm|nomath g2"
SHAPES="${2:-10,4 4,2 20,4 32,4 10,8 32,8 10,12 10,16 20,16 32,16}"
for sh in $SHAPES; do
  k=${sh%,*}; m=${sh#*,}
  timeout -k 10 200 "$R/tools/kbench" $k $m 1048576 256 5 10 > "$OUT/kbench_${k}_${m}.log" 2>&1 || exit $?
  grep -vE "^RS|variant" "$OUT/kbench_${k}_${m}.log" | sed "s/^/RS($k,$m) /"
done
