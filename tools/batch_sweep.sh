# Small-object e2e: per-object calls vs rs_encode_batch / rs_reconstruct_batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/batch; rm -f gpurun_out/batch/sweep.jsonl
for L in 4096 65536 262144; do
  for T in 1 8; do
    timeout -k 10 60 tools/e2e_native 16 4 $L $T 1.5 0,5,16,19 >> gpurun_out/batch/sweep.jsonl || exit 1
    for NB in 64 1024; do
      CALLFS_E2E_BATCH=$NB timeout -k 10 60 tools/e2e_native 16 4 $L $T 1.5 0,5,16,19 >> gpurun_out/batch/sweep.jsonl || exit 1
    done
  done
done
echo batch sweep done
