set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --shard-bytes 6710887 --stripes 256 --cpu-seconds 0 > gpurun_out/bench_cfg1.log 2>&1 || exit $?
bash tools/profile.sh cfg1 --shard-bytes 6710887 --stripes 256 --copy-ceiling 0 || exit $?
timeout -k 10 300 python3 tools/decode_sweep.py --shard-bytes 6710887 --stripes 128 --patterns "enc;;0,1,2,3;0,3,7,12;10,11,12,13" > gpurun_out/decode_cfg2.jsonl 2>&1 || exit $?
echo ok
