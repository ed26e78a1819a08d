# CPU port vs GPU (shim path) per-call encode rate by object size, one request thread.
# Output: gpurun_out/crossover.jsonl. Usage on the GPU box: bash tools/crossover.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/crossover.jsonl; rm -f $O
for km in "10 4" "16 4"; do
  for L in 65536 262144 1048576 4194304 16777216 67108864; do
    for th in 1 16; do timeout -k 10 30 tests/perf/cpu_port_native $km $L $th 1.0 >> $O || exit 1; done
    CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native $km $L 1 1.0 >> $O || exit 1
  done
done
echo ok
