# Counter table of the bit-sliced kernels against the nibble-table kernel on wide shapes
# (what binds each): per (shape, form) a kernel trace and PMC passes of tools/plan_run.py.
# Product library. Usage: bash tools/pmc_bs.sh <tag> <shape> <order> [<order> ...]
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="$1"; SH="$2"; shift 2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
[ -f "$OUT/../avail.txt" ] || timeout -k 10 120 rocprofv3 --list-avail > "$OUT/../avail.txt" 2>&1 || true
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
PB="GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
IC=$(grep -o "SQC_ICACHE_[A-Z_]*" "$OUT/../avail.txt" | sort -u | grep -E "^SQC_ICACHE_(MISSES|HITS|REQ)$" | head -3 | tr '\n' ' ')
for o in "$@"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$o" -o run -- \
    python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 30 > "$OUT/trace_$o.log" 2>&1 || { echo "trace $o rc=$?"; exit 1; }
  for p in A B C; do
    eval "C=\$P$p"
    [ "$p" = C ] && C="$IC"
    [ -z "$C" ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${o}_$p" -o pmc -- \
      python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 8 > "$OUT/pmc_${o}_$p.log" 2>&1
    rc=$?
    case $rc in 0) ;; *) echo "pass $p of $o rc=$rc: stop"; tail -3 "$OUT/pmc_${o}_$p.log"; exit $rc ;; esac
  done
  echo "$o ok"
done
