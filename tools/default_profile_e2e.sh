# CallFS server default profile RS(4,2) (config/loader.go:301-304) end to end through the
# C ABI: pageable (staged) and rs_host_alloc (zero-copy) buffers, 1 and 8 request
# threads, decode erasing one data and one parity shard; CPU port beside it.
# Output: gpurun_out/e2e_rs4_2.jsonl. Usage: bash tools/default_profile_e2e.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/e2e_rs4_2.jsonl; rm -f $O
for L in 1048576 16777216 67108864 268435456; do
  for th in 1 8; do
    echo "{\"mode\": \"staged\", \"threads\": $th}" >> $O
    CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 4 2 $L $th 1.0 1,4 >> $O || exit 1
    echo "{\"mode\": \"pinned\", \"threads\": $th}" >> $O
    CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 4 2 $L $th 1.0 1,4 >> $O || exit 1
  done
  for th in 1 16; do timeout -k 10 30 tests/perf/cpu_port_native 4 2 $L $th 1.0 >> $O || exit 1; done
done
echo ok
