# configs[4]: RS(16,4) encode + reconstruct (erase {0,5,16,19}) over 4 KiB-64 MiB objects,
# host memory in and out (pinned H2D/D2H), staged (pageable) and zero-copy (rs_host_alloc)
# buffers, 1 and 8 request threads. Output: gpurun_out/cfg4_e2e.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/cfg4_e2e.jsonl; rm -f $O
for L in 4096 16384 65536 262144 1048576 4194304 16777216 67108864; do
  for th in 1 8; do
    echo "{\"mode\": \"staged\", \"threads\": $th}" >> $O
    CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 16 4 $L $th 0.8 0,5,16,19 >> $O || exit 1
    echo "{\"mode\": \"pinned\", \"threads\": $th}" >> $O
    CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 16 4 $L $th 0.8 0,5,16,19 >> $O || exit 1
  done
done
echo ok
