# The production dispatch (launch_apply) against the same kernel launched directly
# (kbench "lds ord g2" = LdsG2Policy), three separate processes, bench shape.
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-pvd}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
for rep in 1 2 3; do
  KB_ORD=1 KB_KEEP="lds ord g2|lds ord consec" timeout -k 10 200 "$R/tools/kbench" 10 4 1048576 256 7 10 > "$OUT/rep$rep.log" 2>&1 || exit $?
  grep -E "^(prod|lds ord)" "$OUT/rep$rep.log" | sed "s/^/rep$rep /"
done
cd "$R" && timeout -k 10 300 python3 tools/decode_sweep.py > "$OUT/decode_sweep.jsonl" 2>&1 || exit $?
head -3 "$OUT/decode_sweep.jsonl" | cut -c60-200
