# One large object per call, columns split over 1/2/4 lanes of one device.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/split; rm -f gpurun_out/split/sweep.jsonl
for W in 1 2 4; do
  for L in 268435456 1073741824; do
    CALLFS_RS_SPLIT_WAYS=$W timeout -k 10 60 tools/e2e_native 10 4 $L 1 2.0 0,1,2,3 | sed "s/^{/{\"split_ways\": $W, /" >> gpurun_out/split/sweep.jsonl || exit 1
    CALLFS_E2E_ENCODER=1 CALLFS_RS_SPLIT_WAYS=$W timeout -k 10 60 tools/e2e_native 10 4 $L 1 2.0 0,1,2,3 | sed "s/^{/{\"split_ways\": $W, /" >> gpurun_out/split/sweep.jsonl || exit 1
  done
done
echo split sweep done
