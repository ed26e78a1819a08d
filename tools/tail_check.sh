set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_quick.sh q_tail1 || exit $?
bash tools/wave_tiling_probe.sh wtp_r02b || exit $?
timeout -k 10 400 python3 tools/decode_sweep.py --tune 1 --patterns "enc;;5;0,1,2,3" --shard-bytes 6710887 --stripes 128 > gpurun_out/q_tail1/cfg2.jsonl 2>&1 || exit $?
cut -c1-230 gpurun_out/q_tail1/cfg2.jsonl
