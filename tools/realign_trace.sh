# Which kernels the production dispatch launches for a misaligned Split-layout batch,
# and how long each takes (rocprofv3 kernel trace of tools/kbench, prod dispatch only).
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-rtrace}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export KB_KEEP="__none__"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
  "$R/tools/kbench" 10 4 6710887 64 3 10 1 > "$OUT/kbench.log" 2>&1 || exit $?
cut -c1-160 "$OUT/kt/kt_kernel_stats.csv"
