# The bit-sliced kernel's generator knobs (prefetch depth, waves-per-SIMD floor, block size)
# over a few shapes: one tools/bs_probe.py process per setting. Usage: bash tools/bs_params_r06.sh <tag>
set -o pipefail
T=${1:-bsparams}; O=gpurun_out/r06/$T; mkdir -p $O
S="--shape 32,16,1048576,64 --shape 20,16,262144,384 --shape 32,8,2097152,64 --shape 10,4,1048576,256 --shape 16,8,1048576,256"
for cfg in "2 2 256" "1 2 256" "3 2 256" "4 2 256" "2 3 256" "2 4 256" "2 2 512" "2 2 128" "3 2 512"; do
  set -- $cfg
  CALLFS_RS_BS_PREFETCH=$1 CALLFS_RS_BS_WAVES=$2 CALLFS_RS_BS_BLOCK=$3 CALLFS_RS_JIT_CACHE=0 \
    timeout -k 10 300 python3 -u tools/bs_probe.py --orders bs-g2,bs-g8,bs-q8 --rounds 2 $S \
    | sed "s/^{/{\"pf\": $1, \"waves\": $2, \"block\": $3, /" >> $O/params.jsonl || exit $?
done
