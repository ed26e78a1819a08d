# Verify rows' compare loads issued N shards before the end of the input loop vs after it:
# kbench builds alternated on one box. The builds came from the CALLFS_VERIFY_PREFETCH
# macro of that time (tools/kbench_vpfN with -DCALLFS_VERIFY_PREFETCH=N; now
# Policy::VPF in rs_apply.hpp). Usage: VPF_BUILDS="kbench kbench_vpf4" bash
# tools/verify_prefetch_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-vpf}"; mkdir -p "$OUT"
export KB_KEEP="__none__"
for i in 1 2 3; do
  for b in ${VPF_BUILDS:-kbench kbench_vpf2 kbench_vpf4}; do
    for vm in 0xE 0xF 0x0; do
      KB_VERIFY=$vm timeout -k 10 120 "$R/tools/$b" 10 4 1048576 256 5 10 > "$OUT/${b}_${vm}_$i.log" 2>&1 || exit $?
      echo "$b verify=$vm run $i: $(grep '^prod dispatch' "$OUT/${b}_${vm}_$i.log")"
    done
  done
done
