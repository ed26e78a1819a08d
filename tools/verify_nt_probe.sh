# Verify rows' compare loads: plain loads vs non-temporal loads (now production), two
# kbench builds alternated on one box (tools/kbench_vnt was built with the non-temporal
# load while tools/kbench had the plain one; rs_apply.hpp no longer has the switch).
# Usage: bash tools/verify_nt_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-vnt}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_KEEP="__none__"
for i in 1 2 3; do
  for b in kbench kbench_vnt; do
    for vm in 0xE 0xF 0x0; do
      KB_VERIFY=$vm timeout -k 10 120 "$R/tools/$b" 10 4 1048576 256 5 10 > "$OUT/${b}_${vm}_$i.log" 2>&1 || exit $?
      echo "$b verify=$vm run $i: $(grep '^prod dispatch' "$OUT/${b}_${vm}_$i.log")"
    done
  done
done
