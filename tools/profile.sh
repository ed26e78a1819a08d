# rocprofv3 passes for the bench workload. Usage: bash tools/profile.sh <tag> [bench args]
# 1) --kernel-trace --stats  2) --pmc FETCH_SIZE  3) --pmc WRITE_SIZE (separate passes)
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-r01}"; shift
OUT="$R/gpurun_out/prof_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
  python3 "$R/bench.py" --cpu-seconds 0 --ceiling 0 --layout-ab 0 "$@" > "$OUT/bench_kt.log" 2>&1 || exit $?
echo "kt ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --ceiling 0 --layout-ab 0 "$@" > "$OUT/bench_fetch.log" 2>&1 || exit $?
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --ceiling 0 --layout-ab 0 "$@" > "$OUT/bench_write.log" 2>&1 || exit $?
echo "write ok"
find "$OUT" -name "*.csv" | head -20
