# Round 5's 40 seeded io.ReadAll one-shard decodes (profiles/r05/tiles/random_readall_dec1_*;
# shapes in tools/readall_dec1_shapes.txt), rule against tuner, decode into fresh buffers, on
# the current build. Usage: bash tools/readall_dec1_r06.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O="gpurun_out/${1:-readall_dec1}"; mkdir -p "$O"
A=(); while read -r s; do [ -n "$s" ] && A+=(--shape "$s"); done < tools/readall_dec1_shapes.txt
timeout -k 10 1000 python3 -u tools/ceiling_sweep.py --tune 1 --fresh 1 --only prod,tuned --rounds 2 "${A[@]}" > "$O/sweep.jsonl" 2> "$O/sweep.err" || exit $?
echo ok
