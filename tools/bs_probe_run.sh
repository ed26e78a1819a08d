set -o pipefail
O=gpurun_out/r06/bs1; mkdir -p $O
export CALLFS_RS_BITSLICE_LOG=1 CALLFS_RS_JIT_CACHE=$PWD/gpurun_out/r06/jit
timeout -k 10 500 python3 -u tools/bs_probe.py --orders bs,bs-q8,bs-x32,bs-g2 \
  --shape 32,16,1048576,64 --shape 20,16,1048576,96 --shape 10,16,1048576,128 \
  --shape 32,8,2097152,64 --shape 16,8,1048576,256 --shape 20,16,1048576,96,0+1+2+3+4+5+6+7+20+21+22+23+24+25+26+27 \
  > $O/probe.jsonl 2> $O/probe.err
