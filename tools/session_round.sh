# One gpurun call: full GPU round (tests, smoke, bench, rocprofv3 passes), then the LDS
# lookup-rate probe and the configs[4] end-to-end sweep. Usage: bash tools/session_round.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-r03s4}"; cd "$R"
bash tools/gpu_round.sh "$TAG" || exit $?
timeout -k 10 120 tools/lds_rate 2000 > "gpurun_out/$TAG/lds_rate.txt" 2>&1 || exit $?
echo "lds_rate ok"; cat "gpurun_out/$TAG/lds_rate.txt"
bash tools/cfg4_e2e.sh && mv gpurun_out/cfg4_e2e.jsonl "gpurun_out/$TAG/" && echo "cfg4 ok"
