# Wide groups (R = 12, 16): the production LDS kernel (16-byte entries) against the hybrid
# row split of tools/kbench (rows 0..7 through 8-byte LDS entries, the rest v_perm on the
# VALU), timed interleaved, then PMC counters of each alone (LDS-array busy, VALU busy,
# effective clock). Usage: bash tools/hybrid_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-hybrid}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for sh in "32 16" "20 16" "10 16" "10 12"; do
  unset KB_HYBRID KB_HYBRID_FIRST
  set -- $sh; k=$1; m=$2; B=$(( k >= 20 ? 128 : 256 ))
  KB_HYBRID=1 KB_KEEP="hybrid" timeout -k 10 150 "$R/tools/kbench" $k $m 1048576 $B 5 10 > "$OUT/time_${k}_${m}.log" 2>&1 || exit $?
  grep -E "prod dispatch|hybrid|MISMATCH" "$OUT/time_${k}_${m}.log" | sed "s/^/RS($k,$m) /"
  for v in prod hybrid; do
    for p in A B; do
      eval "C=\$P$p"
      if [ $v = hybrid ]; then export KB_HYBRID=1 KB_HYBRID_FIRST=1; else unset KB_HYBRID KB_HYBRID_FIRST; fi
      KB_KEEP="__none__" timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${v}_${k}_${m}_$p" -o pmc -- \
        "$R/tools/kbench" $k $m 1048576 $B 1 3 > "$OUT/pmc_${v}_${k}_${m}_$p.log" 2>&1
      rc=$?
      case $rc in 0) ;; 124|134|137|139) echo "pass $p of $v $k,$m ended rc=$rc: stop"; exit $rc ;;
        *) echo "pass $p of $v $k,$m failed rc=$rc"; tail -3 "$OUT/pmc_${v}_${k}_${m}_$p.log" ;; esac
    done
  done
done
unset KB_HYBRID KB_HYBRID_FIRST
