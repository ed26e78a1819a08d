# Triple loads in every tile order (tools/kbench KB_TRIORD) beside the nibble kernel's
# orders (KB_ORD) on the few-input large-shard shapes. Usage: bash tools/triord_probe.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-triord}"; mkdir -p "$OUT"; : > "$OUT/summary.txt"
for sh in "4 2 16777216 42 256 0" "4 2 16777216 42 256 4096" "4 2 8388608 85 256 0" "6 3 16777216 28 256 0" "4 2 33554432 21 256 0"; do
  set -- $sh; k=$1; m=$2; S=$3; B=$4; al=$5; pad=$6
  KB_TRIORD=1 KB_ORD=1 KB_KEEP="tri ord|lds ord consec|lds ord q8|lds ord q16" timeout -k 10 200 tools/kbench $k $m $S $B 4 10 $al $pad \
    > "$OUT/kb_${k}_${m}_${S}_$pad.log" 2>&1 || exit $?
  grep -E "prod dispatch|ord" "$OUT/kb_${k}_${m}_${S}_$pad.log" | sed "s/^/RS($k,$m) S=$S pad=$pad /" | tee -a "$OUT/summary.txt"
done
