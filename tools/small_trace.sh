# Where a small host-memory call's time goes: kernel trace (+ HIP API trace) of
# single-thread 4 KiB RS(16,4) calls (encoder path, then decode), staged path
# (CALLFS_RS_SMALL_MAX_BYTES=0) and one-dispatch small path. Usage: bash tools/small_trace.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-smalltrace}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export CALLFS_E2E_ENCODER=1
for lim in 0 2097152; do
  CALLFS_RS_SMALL_MAX_BYTES=$lim timeout -k 10 60 "$R/tools/e2e_native" 16 4 4096 1 1.0 0,5,16,19 > "$OUT/plain_$lim.jsonl" 2>&1 || exit $?
  CALLFS_RS_SMALL_MAX_BYTES=$lim timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$OUT/trace_$lim" -o tr -- \
    "$R/tools/e2e_native" 16 4 4096 1 0.3 0,5,16,19 > "$OUT/traced_$lim.jsonl" 2>&1 || exit $?
done
echo ok
