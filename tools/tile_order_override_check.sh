# bench.py under each CALLFS_RS_TILE_ORDER override (device round trip checked by bench.py itself)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ovr
for o in consecutive g8 g2 q8 q16; do
  CALLFS_RS_TILE_ORDER=$o timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --ceiling 0 > gpurun_out/ovr/$o.log 2>&1 || exit $?
  echo "$o $(tail -1 gpurun_out/ovr/$o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"])')"
done
