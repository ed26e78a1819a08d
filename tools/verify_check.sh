# GPU tests, then decode per erasure pattern (rule order) on the bench shape and the
# configs[2] shape. Usage: bash tools/verify_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG="${1:-vchk}"; OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
bash tools/gpu_quick.sh "$TAG" || exit $?
timeout -k 10 300 python3 tools/decode_sweep.py > "$OUT/decode_bench_shape.jsonl" 2>&1 || exit $?
timeout -k 10 300 python3 tools/decode_sweep.py --shard-bytes 6710887 --stripes 128 > "$OUT/decode_cfg2.jsonl" 2>&1 || exit $?
grep '^{' "$OUT/decode_bench_shape.jsonl" "$OUT/decode_cfg2.jsonl" | python3 -c "
import json,sys
for ln in sys.stdin:
    f,j=ln.split(':',1); d=json.loads(j); print(f.split('/')[-1], d['plan'], d['frac_8TBs'])"
