# 1 MiB objects with many inputs or 8 rows in the planar layout: every tile order of the
# ring-of-three and triple forms (tools/order_ab.py). Usage: bash tools/small_r8_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-smallr8}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python3 -u tools/order_ab.py --rounds 3 --orders consecutive,g2,g8,x32,tri,tri-g2,tri-x32,tri-x8 \
  --shape 32,8,32768,3276,-,planar --shape 20,4,52429,3413,-,planar --shape 10,8,104858,2275,-,planar \
  --shape 32,8,32768,3276,-,pitch --shape 16,8,65536,2048,-,planar --shape 12,8,87382,2048,-,planar \
  > "$O/ab.jsonl" 2>&1 || exit $?
echo "ab ok"
