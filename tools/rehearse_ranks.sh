# N > 1 launch rehearsal on a 1-GPU box (ranks share the device, LOCAL_RANK % device_count):
# the driver's torchrun line at N = 4 (weak, default workload) and the configs[3] column
# split (1 GiB objects, strong) at N = 1 and 4. Usage: bash tools/rehearse_ranks.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-ranks}"; mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 4 --steps 10 --warmup 2 > "$OUT/weak4.log" 2>&1 || exit $?
grep '^{' "$OUT/weak4.log" | cut -c1-160
timeout -k 10 300 python3 bench.py --object-bytes 1073741824 --steps 5 --warmup 1 --cpu-seconds 0 > "$OUT/obj1.log" 2>&1 || exit $?
grep '^{' "$OUT/obj1.log" | cut -c1-160
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 4 --object-bytes 1073741824 --steps 5 --warmup 1 > "$OUT/obj4.log" 2>&1 || exit $?
grep '^{' "$OUT/obj4.log" | cut -c1-160
