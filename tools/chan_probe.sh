# Memory-side (L2 -> fabric) request, latency and stall counters for the configs[1] encode and
# decode against the 1 / 2 MiB shapes ("TCC channel counters";
# rocprofv3 reports each summed over the 16 channels x 8 XCDs). Lists the counters and their
# dimensions, then one --pmc pass per counter group over tools/ceiling_sweep.py (the plan's
# launch and its read-alone / write-alone streams).
# Usage: [SHAPES='k,m,S,B,erase,layout[,order] ...'] bash tools/chan_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-chan}"
OUT="$R/gpurun_out/chan_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/list.txt" 2>&1 || exit $?
# SHAPES overrides the shape list (tools/ceiling_sweep.py specs, space-separated)
SHAPES="${SHAPES:-10,4,2097152,192,-,planar 10,4,6710887,64,-,planar 10,4,1048576,384,-,planar 10,4,6710887,64,0+1+2+3,planar}"
SH=""; for x in $SHAPES; do SH="$SH --shape $x"; done
i=0
# pass 1: requests and requests in flight (average latency = LEVEL / REQ); pass 2: stalls;
# pass 3: requests that reach DRAM (the rest are served by the Infinity Cache)
G=GRBM_GUI_ACTIVE
for C in "TCC_EA0_WRREQ TCC_EA0_RDREQ TCC_EA0_WRREQ_LEVEL TCC_EA0_RDREQ_LEVEL $G" \
         "TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_STALL TCC_TAG_STALL $G" \
         "TCC_EA0_WRREQ_DRAM TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ TCC_EA0_RDREQ $G"; do
  i=$((i + 1))
  for c in $C; do grep -qw "$c" "$OUT/list.txt" || { echo "no $c"; continue 2; }; done
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o p$i -- \
    python3 "$R/tools/ceiling_sweep.py" $SH --fresh 1 --only prod,read,write --rounds 1 --reps 3 \
    > "$OUT/p$i.log" 2>&1 || exit $?
  echo "pass $i ok"
done
find "$OUT" -name "*.csv" | head
