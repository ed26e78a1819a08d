# Counter table of kernel forms on one shape (what binds R 5..8): per form a kernel trace
# (time) and two PMC passes (tools/plan_run.py under rocprofv3), A/B build of the library.
# Usage: bash tools/pmc_forms.sh <tag> <shape> <order> [<order> ...]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="$1"; SH="$2"; shift 2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
# the A/B build is not pushed: built here on demand (build/ab/, tools/callfs_rs_ab.h)
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
export CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so"
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for o in "$@"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$o" -o run -- \
    python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 30 > "$OUT/trace_$o.log" 2>&1 || { echo "trace $o rc=$?"; exit 1; }
  for p in A B; do
    eval "C=\$P$p"
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${o}_$p" -o pmc -- \
      python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 8 > "$OUT/pmc_${o}_$p.log" 2>&1
    rc=$?
    case $rc in 0) ;; *) echo "pass $p of $o rc=$rc: stop"; tail -3 "$OUT/pmc_${o}_$p.log"; exit $rc ;; esac
  done
  echo "$o ok"
done
