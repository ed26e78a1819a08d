# Zero-copy concurrency probes: is the 8-thread loss on large pinned
# objects concurrency, pinned footprint, or per-call allocation? RS(4,2) 256 MiB through
# the encoder path (rs_encode on rs_host_alloc buffers), decode erasing {1,4}.
# Usage: bash tools/zerocopy_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-zc}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
E="$R/tools/e2e_native"
{ echo "nproc $(nproc)"; cat /sys/class/drm/card*/device/numa_node 2>/dev/null | tr '\n' ' '; echo;
  ls /sys/devices/system/node | grep node | tr '\n' ' '; echo; grep -i huge /proc/meminfo;
  cat /sys/kernel/mm/transparent_hugepage/enabled; ulimit -l; } > "$OUT/host_info.txt" 2>&1
run() {  # name env... -- args
  local name=$1; shift
  echo "{\"case\": \"$name\"}" >> "$OUT/zc.jsonl"
  env "$@" >> "$OUT/zc.jsonl" 2>> "$OUT/zc.err"
  local rc=$?; tail -1 "$OUT/zc.jsonl"; return $rc
}
export CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1
for rep in a b; do
run t1_$rep timeout -k 10 120 $E 4 2 268435456 1 6 1,4 || exit $?
run t8_$rep timeout -k 10 120 $E 4 2 268435456 8 6 1,4 || exit $?
done
run t8_serial CALLFS_E2E_SERIAL=1 timeout -k 10 120 $E 4 2 268435456 8 6 1,4 || exit $?
run t1_extra12g CALLFS_E2E_EXTRA_PINNED_MIB=12288 timeout -k 10 180 $E 4 2 268435456 1 6 1,4 || exit $?
run t8_extra12g CALLFS_E2E_EXTRA_PINNED_MIB=12288 timeout -k 10 180 $E 4 2 268435456 8 6 1,4 || exit $?
run t2 timeout -k 10 120 $E 4 2 268435456 2 6 1,4 || exit $?
run t4 timeout -k 10 120 $E 4 2 268435456 4 6 1,4 || exit $?
run t8_32mib timeout -k 10 120 $E 4 2 33554432 8 6 1,4 || exit $?
run t1_fresh CALLFS_E2E_FRESH=1 timeout -k 10 120 $E 4 2 268435456 1 6 1,4 || exit $?
run t8_fresh CALLFS_E2E_FRESH=1 timeout -k 10 120 $E 4 2 268435456 8 6 1,4 || exit $?
run rs10_4_t8_256m timeout -k 10 120 $E 10 4 268435456 8 6 0,1,2,3 || exit $?
run rs10_4_t1_256m timeout -k 10 120 $E 10 4 268435456 1 6 0,1,2,3 || exit $?
cd /tmp && export TMPDIR=/tmp
for t in 1 8; do
  timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d "$OUT/trace_t$t" -o tr -- $E 4 2 268435456 $t 3 1,4 > "$OUT/trace_t$t.log" 2>&1 || exit $?
done
echo done
