# The triple-load forms (plain kernel, unaligned 16-B accesses) against the realigning
# kernel on misaligned shards: upstream Split layouts (contiguous 'split' and the io.ReadAll
# body 'readall'), encode and decodes, beside the same shapes at the 256-B pitch.
# Usage: bash tools/unaligned_tri_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-utri}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
ORD=realign-x32,realign,tri-x32,tri-g2,tri-q8,tri-x8,tri,g2,x32
run() {  # name, shapes...
  local n=$1; shift
  timeout -k 10 500 python3 -u tools/order_ab.py --rounds 3 --orders $ORD "$@" > "$O/$n.jsonl" 2>&1 || exit $?
  echo "$n ok"
}
S1="10,4,6710887,64 4,2,1048577,512 6,3,1048577,256 10,8,1048577,256 12,4,5592406,64 5,3,209716,1024"
S2="10,4,104858,1024 6,3,174763,2048 12,4,87382,1024 20,4,52429,1024 10,8,104858,1024 8,4,131072,1024 16,4,65536,1024 4,2,262145,2048"
A=(); for s in $S1 $S2; do A+=(--shape "$s,-,split"); done; run split_enc "${A[@]}"
A=(); for s in $S1 $S2; do A+=(--shape "$s,-,readall"); done; run readall_enc "${A[@]}"
A=(); for s in $S2; do A+=(--shape "$s,-,pitch"); done; run pitch_enc "${A[@]}"
# decodes: four / one data erasures (misaligned outputs), Split layouts
A=(); for s in 10,4,6710887,64 10,4,104858,1024; do
  A+=(--shape "$s,0+1+2+3,split" --shape "$s,5,split" --shape "$s,0+1+2+3,readall"); done
A+=(--shape 6,3,1048577,256,0+1+2,split --shape 6,3,1048577,256,2,split)
run decode "${A[@]}"
