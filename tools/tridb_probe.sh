# Triple-loop forms against each other (tools/kbench KB_TRIDB): production WIX 2, zeros for
# loads past K (WIX 4), two register sets without conditional loads (WIX 3, at the
# compiler's 81 VGPRs / 5 waves and at <= 80 / 6 waves). Usage: bash tools/tridb_probe.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-tridb}"; mkdir -p "$OUT"; : > "$OUT/summary.txt"
for sh in "4 2 1048576" "4 2 4194304" "4 2 16777216" "4 2 262144" "6 3 1048576" "6 3 4194304" "6 3 174763" \
          "10 4 1048576" "10 4 16777216" "8 4 2097152" "12 4 1048576" "8 8 2097152" "10 8 1677722"; do
  set -- $sh; k=$1; m=$2; S=$3
  B=$(( (4 << 30) / (S * (k + m)) ))
  KB_TRIDB=1 KB_KEEP="tri2|tri4|tridb|pairdb" timeout -k 10 200 tools/kbench $k $m $S $B 4 10 > "$OUT/kb_${k}_${m}_$S.log" 2>&1 || exit $?
  grep -E "prod dispatch|tri|MISMATCH" "$OUT/kb_${k}_${m}_$S.log" | sed "s/^/RS($k,$m) S=$S /" | tee -a "$OUT/summary.txt"
done
