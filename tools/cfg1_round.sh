# configs[1]/[2] shape (RS(10,4), 256 objects of 64 MiB = 6,710,887-B shards, 24 GB
# resident): bench line + rocprofv3 kernel trace / FETCH / WRITE passes.
# Usage: bash tools/cfg1_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG="${1:-cfg1}"; mkdir -p "gpurun_out/$TAG"
timeout -k 10 400 python3 bench.py --shard-bytes 6710887 --stripes 256 --steps 10 --warmup 2 --cpu-seconds 5 \
  > "gpurun_out/$TAG/bench.log" 2>&1 || exit $?
tail -1 "gpurun_out/$TAG/bench.log" | cut -c1-300
bash tools/profile.sh "$TAG" --shard-bytes 6710887 --stripes 256 --steps 5 --warmup 1
