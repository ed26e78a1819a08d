# rocprofv3 --pmc passes over tools/ceiling_sweep.py (production launch only), one process
# per shape and counter set. Usage: bash tools/pmc_sweep.sh <tag> <shape> [<shape> ...]
# Counter sets (each its own pass, under a kill timer): FETCH_SIZE; WRITE_SIZE; TCC
# request sizes; SQ LDS/VALU activity; memory-side read queue level and DRAM credit
# stalls; write queue level and stalls (PASSES="4 5" picks sets). Summarise with
# tools/pmc_sweep_table.py.
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="$1"; shift
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
SETS=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_CYCLE_sum")
PASSES=${PASSES:-"0 1 2 3 4 5"}
i=0
for sh in "$@"; do
  i=$((i+1))
  for s in $PASSES; do
    d="$OUT/s${i}_p$s"
    timeout -s KILL 90 rocprofv3 --pmc ${SETS[$s]} --output-format csv -d "$d" -o pmc -- \
      python3 "$R/tools/ceiling_sweep.py" --rounds 1 --reps 3 --only prod --shape "$sh" > "$d.log" 2>&1
    rc=$?
    case $rc in 0) ;; 124|134|137|139) echo "pass $s of $sh ended rc=$rc: stop"; exit $rc ;;
      *) echo "pass $s of $sh failed rc=$rc"; tail -3 "$d.log" ;; esac
  done
  echo "$sh" > "$OUT/s${i}.shape"
  echo "shape $sh done"
done
