# Live-ceiling table over the shapes VERDICT r02 names (tools/ceiling_sweep.py).
# Usage: bash tools/ceiling_round.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-ceil}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
run() {  # name, shapes...
  local name=$1; shift
  local args=()
  for s in "$@"; do args+=(--shape "$s"); done
  timeout -k 10 300 python3 -u tools/ceiling_sweep.py --tune 1 "${args[@]}" > "$OUT/$name.jsonl" 2> "$OUT/$name.err" || { echo "$name failed rc=$?"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "$name ok"
}
run bench 10,4,1048576,256 10,4,1048576,256,none 10,4,1048576,256,0+1+2+3
run one_erasure 10,4,1048576,256,5 10,4,1048576,256,0 10,4,1048576,256,13 10,4,6710887,64,5 10,4,6710887,64,13
run wide 10,12,1048576,256 10,16,1048576,256 20,16,1048576,128 32,16,1048576,64 20,4,1048576,128 32,8,1048576,64
run split 10,4,6710887,64,-,split 10,4,1048577,256,-,split 10,8,1048577,256,-,split 4,2,1048577,512,-,split 12,4,5592406,64,-,split
run small 10,8,104858,2000 6,3,174763,2600 10,4,104858,2900 12,4,87382,2900 10,8,1677722,128 10,4,1677722,180
