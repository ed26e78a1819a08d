set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/e2e
O=gpurun_out/e2e/zc_small.jsonl; rm -f $O
export CALLFS_E2E_PINNED=1
for zc in 0 1099511627776; do
  echo "{\"zc_min\": $zc}" >> $O
  for L in 4096 65536 131072 262144 524288 1048576; do CALLFS_RS_ZERO_COPY_MIN_BYTES=$zc timeout -k 10 60 tools/e2e_native 16 4 $L 1 0.7 0,5,16,19 >> $O || exit 1; done
  for L in 262144 524288 1048576; do CALLFS_RS_ZERO_COPY_MIN_BYTES=$zc timeout -k 10 60 tools/e2e_native 10 4 $L 1 0.7 0,1,2,3 >> $O || exit 1; done
done
echo ok
