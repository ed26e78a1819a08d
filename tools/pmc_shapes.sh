# PMC counters of the production dispatch (tools/kbench, variant 0 only) on the row-group
# shapes furthest below roofline. Usage: bash tools/pmc_shapes.sh <tag>
# Each rocprofv3 --pmc pass runs on its own (<= 8 SQ counters, <= 2 GRBM), under a kill timer.
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-pmc}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
export KB_KEEP="__none__"
SHAPES="10,4 10,8 32,8 20,4 10,12 10,16 20,16 32,16"
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for sh in $SHAPES; do
  k=${sh%,*}; m=${sh#*,}
  timeout -k 10 120 "$R/tools/kbench" $k $m 1048576 256 3 5 > "$OUT/kbench_${k}_${m}.log" 2>&1 || exit $?
  for p in A B; do
    eval "C=\$P$p"
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${k}_${m}_$p" -o pmc -- \
      "$R/tools/kbench" $k $m 1048576 256 1 3 > "$OUT/pmc_${k}_${m}_$p.log" 2>&1
    rc=$?
    case $rc in 0) ;; 124|134|137|139) echo "pass $p of $k,$m ended rc=$rc: stop"; exit $rc ;;
      *) echo "pass $p of $k,$m failed rc=$rc (counter set?)"; tail -3 "$OUT/pmc_${k}_${m}_$p.log" ;; esac
  done
  echo "shape $k,$m done"
done
