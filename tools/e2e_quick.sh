set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/e2e
O=gpurun_out/e2e/coh.jsonl; rm -f $O
for rep in 1 2; do for coh in 0 1; do
  for cfg in "4096 1" "4096 8" "65536 1" "65536 8" "1048576 1" "1048576 8" "16777216 1" "67108864 1"; do
    set -- $cfg
    echo "{\"coherent\": $coh}" >> $O
    if [ $coh = 1 ]; then export CALLFS_RS_PINNED_COHERENT=1; else unset CALLFS_RS_PINNED_COHERENT; fi
    timeout -k 10 60 tools/e2e_native 16 4 $1 $2 0.7 0,5,16,19 >> $O || exit 1
  done
done; done
echo ok
