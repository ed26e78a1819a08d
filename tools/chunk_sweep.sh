# Pipeline chunk-size sweep for the host-memory path (native driver, one thread).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/chunk; rm -f gpurun_out/chunk/sweep.jsonl
for cb in 262144 1048576 4194304 16777216; do
  for L in 1048576 4194304 16777216 67108864; do
    CALLFS_RS_CHUNK_BYTES=$cb timeout -k 10 60 tools/e2e_native 16 4 $L 1 1.0 0,5,16,19 | sed "s/^{/{\"chunk\": $cb, /" >> gpurun_out/chunk/sweep.jsonl || exit 1
  done
  CALLFS_RS_CHUNK_BYTES=$cb timeout -k 10 60 tools/e2e_native 10 4 1073741824 1 2.0 0,1,2,3 | sed "s/^{/{\"chunk\": $cb, /" >> gpurun_out/chunk/sweep.jsonl || exit 1
done
echo chunk sweep done
for L in 1048576 16777216 67108864 1073741824; do
  timeout -k 10 60 tools/e2e_native 10 4 $L 1 2.0 0,1,2,3 >> gpurun_out/chunk/sweep.jsonl || exit 1
  timeout -k 10 60 tools/e2e_native 10 4 $L 8 2.0 0,1,2,3 >> gpurun_out/chunk/sweep.jsonl || exit 1
  CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 10 4 $L 1 2.0 0,1,2,3 >> gpurun_out/chunk/sweep.jsonl || exit 1
  CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 10 4 $L 8 2.0 0,1,2,3 >> gpurun_out/chunk/sweep.jsonl || exit 1
done
echo encoder sweep done
