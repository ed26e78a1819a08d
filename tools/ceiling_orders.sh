# Read-alone / write-alone rates per tile order (tools/ceiling_orders.py) on the configs[1]
# shape and the bench shape. Usage: bash tools/ceiling_orders.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-ceilord}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python3 -u tools/ceiling_orders.py --orders consecutive,g2,g8,q8,q16,x8,x32 \
  --shape 10,4,6710887,256,-,planar --shape 10,4,1048576,256,-,planar \
  --shape 10,4,2097152,128,-,planar --shape 10,4,8388608,32,-,planar \
  --shape 10,4,6710887,256,-,pitch > "$O/ceil_orders.jsonl" 2>&1 || exit $?
echo "ceiling orders ok"
