# Where a small host-memory call's time goes: kernel + memory-copy trace of single-thread
# 4 KiB RS(16,4) calls (encoder path, then decode). Usage: bash tools/small_trace.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-smalltrace}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export CALLFS_E2E_ENCODER=1
timeout -k 10 60 "$R/tools/e2e_native" 16 4 4096 1 1.0 0,5,16,19 > "$OUT/plain.jsonl" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o tr -- \
  "$R/tools/e2e_native" 16 4 4096 1 0.3 0,5,16,19 > "$OUT/traced.jsonl" 2>&1 || exit $?
echo ok
