# Host-memory crossover on the current build: per-call encode and
# degraded decode rate of the GPU path through the C ABI -- pageable buffers (staged, or
# the one-dispatch small path) and rs_host_alloc buffers (zero-copy) -- at 1 and 8
# request threads, against the CPU port of upstream's codec at 1 and 16 threads, for the
# CallFS default RS(4,2) (config/loader.go:300-304) and RS(10,4).
# Output: gpurun_out/<tag>/crossover.jsonl. Usage: bash tools/crossover_r04.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-crossover_r04}"; mkdir -p "$OUT"; O=$OUT/crossover.jsonl; : > $O
for km in "4 2" "10 4"; do
  set -- $km; k=$1; m=$2; er="1,$k"
  for L in 65536 262144 1048576 4194304 16777216 67108864 268435456; do
    for th in 1 16; do
      echo "{\"impl\": \"cpu_port\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      timeout -k 10 30 tests/perf/cpu_port_native $k $m $L $th 0.6 >> $O || exit 1
    done
    for th in 1 8; do
      echo "{\"impl\": \"gpu_staged\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native $k $m $L $th 0.6 $er >> $O || exit 1
      echo "{\"impl\": \"gpu_pinned\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native $k $m $L $th 0.6 $er >> $O || exit 1
    done
  done
done
echo ok
