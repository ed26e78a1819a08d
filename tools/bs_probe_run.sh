# tools/bs_probe.py over a set of shapes on the GPU box. Usage: bash tools/bs_probe_run.sh <tag> <shape>...
set -o pipefail
T=${1:-bs}; shift
O=gpurun_out/r06/$T; mkdir -p $O
export CALLFS_RS_BITSLICE_LOG=1 CALLFS_RS_JIT_CACHE=$PWD/gpurun_out/r06/jit
A=(); for s in "$@"; do A+=(--shape "$s"); done
timeout -k 10 900 python3 -u tools/bs_probe.py ${BS_ARGS:-} --orders ${BS_ORDERS:-bs,bs-q8,bs-x32,bs-g2} "${A[@]}" > $O/probe.jsonl 2> $O/probe.err
