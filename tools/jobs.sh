# GPU-box jobs: the measurement recipes behind profiles/ (one function per job). Run on a
# box through gpurun from the repo root: bash tools/jobs.sh <job> [args]. With no job, lists
# them. Each GPU step has its own time limit and a failing step ends the job (no retries).
# Kept apart: tools/zerocopy_probe.sh (a copy-trace pass) and tools/gpurun_retry.sh (runs
# here, around gpurun).
set -o pipefail
JOBS="$(cd "$(dirname "$0")" && pwd)/$(basename "$0")"

# The driver's bench line on this build, a wide-profile line (RS(20,16), 16 erasures: the
# bit-sliced kernels), and the A/B build's offered-order parity cases (the LDS-DMA ring with
# K below its depth). Usage: bash tools/jobs.sh bench_r06 <tag>
job_bench_r06() {
T=${1:-bench}; O=gpurun_out/r06/$T; mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2> $O/bench.err || exit $?
echo "bench ok"; tail -c 600 $O/bench.log
timeout -k 10 300 python3 -u bench.py --k 20 --m 16 --erase 0,1,2,3,4,5,6,7,20,21,22,23,24,25,26,27 \
  --layout-ab 0 --cpu-seconds 3 > $O/bench_rs20_16.log 2> $O/bench_rs20_16.err || exit $?
echo "wide bench ok"
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null 2> $O/build_ab.err || exit $?
CALLFS_RS_LIB=$PWD/build/ab/libcallfs_rs_ab.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py -k every_offered > $O/pytest_ab.log 2>&1 || exit $?
echo "ab tests ok"; tail -2 $O/pytest_ab.log
}

# The bit-sliced kernel's generator knobs (prefetch depth, waves-per-SIMD floor, block size)
# over a few shapes: one tools/bs_probe.py process per setting. Usage: bash tools/jobs.sh bs_params_r06 <tag>
job_bs_params_r06() {
T=${1:-bsparams}; O=gpurun_out/r06/$T; mkdir -p $O
S="--shape 32,16,1048576,64 --shape 20,16,262144,384 --shape 32,8,2097152,64 --shape 10,4,1048576,256 --shape 16,8,1048576,256"
for cfg in "2 2 256" "1 2 256" "3 2 256" "4 2 256" "2 3 256" "2 4 256" "2 2 512" "2 2 128" "3 2 512"; do
  set -- $cfg
  CALLFS_RS_BS_PREFETCH=$1 CALLFS_RS_BS_WAVES=$2 CALLFS_RS_BS_BLOCK=$3 CALLFS_RS_JIT_CACHE=0 \
    timeout -k 10 300 python3 -u tools/bs_probe.py --orders bs-g2,bs-g8,bs-q8 --rounds 2 $S \
    | sed "s/^{/{\"pf\": $1, \"waves\": $2, \"block\": $3, /" >> $O/params.jsonl || exit $?
done
}

# tools/bs_probe.py over a set of shapes on the GPU box. Usage: bash tools/jobs.sh bs_probe_run <tag> <shape>...
job_bs_probe_run() {
T=${1:-bs}; shift
O=gpurun_out/r06/$T; mkdir -p $O
export CALLFS_RS_BITSLICE_LOG=1 CALLFS_RS_JIT_CACHE=$PWD/gpurun_out/r06/jit
A=(); for s in "$@"; do A+=(--shape "$s"); done
timeout -k 10 900 python3 -u tools/bs_probe.py ${BS_ARGS:-} --orders ${BS_ORDERS:-bs,bs-q8,bs-x32,bs-g2} "${A[@]}" > $O/probe.jsonl 2> $O/probe.err
}

# Bit-sliced orders against the rule over the shapes the rule is fitted on (planar), then the
# io.ReadAll one-shard decodes. Usage: bash tools/jobs.sh bs_sweep_r06 <tag>
job_bs_sweep_r06() {
T=${1:-sweep}
export BS_ORDERS=bs,bs-g2,bs-g8,bs-q8,bs-x32
bash "$JOBS" bs_probe_run $T \
 32,16,65536,1024 32,16,262144,256 32,16,1048576,64 32,16,4194304,16 \
 20,16,65536,1536 20,16,262144,384 20,16,1048576,96 20,16,4194304,24 \
 10,16,262144,512 10,16,1048576,128 10,16,4194304,32 10,12,1048576,128 20,9,1048576,128 \
 32,8,524288,256 32,8,2097152,64 16,8,262144,1024 16,8,1048576,256 16,8,4194304,64 12,8,1048576,256 \
 10,8,6710887,32 10,8,1048576,256 10,8,262144,1024 8,8,1048576,256 8,6,1048576,256 10,6,1048576,256 \
 32,4,1048576,128 24,4,1048576,160 20,4,3355444,64 16,4,4194304,64 10,4,1048576,256 && \
BS_ARGS="--layout readall --fresh 1" bash "$JOBS" bs_probe_run ${T}_readall \
 10,8,553574,512,1 10,8,122190,2048,1 8,8,312855,1024,1 10,8,1048576,256,1 16,8,1048576,256,1 10,4,104858,2048,1 \
 10,8,6710887,32,1 10,4,1048576,256,1
}

# Read-alone / write-alone rates per tile order (tools/ceiling_orders.py) on the configs[1]
# shape and the bench shape. Usage: bash tools/jobs.sh ceiling_orders <tag>
job_ceiling_orders() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-ceilord}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python3 -u tools/ceiling_orders.py --orders consecutive,g2,g8,q8,q16,x8,x32 \
  --shape 10,4,6710887,256,-,planar --shape 10,4,1048576,256,-,planar \
  --shape 10,4,2097152,128,-,planar --shape 10,4,8388608,32,-,planar \
  --shape 10,4,6710887,256,-,pitch > "$O/ceil_orders.jsonl" 2>&1 || exit $?
echo "ceiling orders ok"
}

# configs[1]/[2] shape (RS(10,4), S = 6,710,887, planar) against neighbouring shard sizes:
# every tile order and kernel form the plan offers (tools/order_ab.py), to tell a shard-size
# effect from an order effect. Usage: bash tools/jobs.sh cfg12_orders <tag>
job_cfg12_orders() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-cfg12o}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
ORD=consecutive,g2,q8,q16,x8,x32,tri,tri-g2,tri-q8,tri-q16,tri-x8,tri-x32
A=()
for s in 10,4,6710887,45,- 10,4,6710887,45,0+1+2+3 10,4,6710880,45,- 10,4,8388608,36,- \
         10,4,4194304,73,- 10,4,2097152,146,- 10,4,1048576,292,- 10,4,6710887,256,-; do
  A+=(--shape "$s,planar")
done
timeout -k 10 900 python3 -u tools/order_ab.py --rounds 3 --orders "$ORD" "${A[@]}" \
  > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
}

# configs[4]: RS(16,4) encode + reconstruct (erase {0,5,16,19}) over 4 KiB-64 MiB objects,
# host memory in and out (pinned H2D/D2H), staged (pageable) and zero-copy (rs_host_alloc)
# buffers, 1 and 8 request threads. Output: gpurun_out/cfg4_e2e.jsonl
job_cfg4_e2e() {
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/cfg4_e2e.jsonl; rm -f $O
for L in 4096 16384 65536 262144 1048576 4194304 16777216 67108864; do
  for th in 1 8; do
    echo "{\"mode\": \"staged\", \"threads\": $th}" >> $O
    CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 16 4 $L $th 0.8 0,5,16,19 >> $O || exit 1
    echo "{\"mode\": \"pinned\", \"threads\": $th}" >> $O
    CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 16 4 $L $th 0.8 0,5,16,19 >> $O || exit 1
  done
done
echo ok
}

# Memory-side (L2 -> fabric) request, latency and stall counters for the configs[1] encode and
# decode against the 1 / 2 MiB shapes ("TCC channel counters";
# rocprofv3 reports each summed over the 16 channels x 8 XCDs). Lists the counters and their
# dimensions, then one --pmc pass per counter group over tools/ceiling_sweep.py (the plan's
# launch and its read-alone / write-alone streams).
# Usage: [SHAPES='k,m,S,B,erase,layout[,order] ...'] bash tools/jobs.sh chan_probe <tag>
job_chan_probe() {
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
}

# Host-memory crossover on the current build: per-call encode and
# degraded decode rate of the GPU path through the C ABI -- pageable buffers (staged, or
# the one-dispatch small path) and rs_host_alloc buffers (zero-copy) -- at 1 and 8
# request threads, against the CPU port of upstream's codec at 1 and 16 threads, for the
# CallFS default RS(4,2) (config/loader.go:300-304) and RS(10,4).
# Output: gpurun_out/<tag>/crossover.jsonl. Usage: bash tools/jobs.sh crossover_r04 <tag>
job_crossover_r04() {
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-crossover_r04}"; mkdir -p "$OUT"; O=$OUT/crossover.jsonl; : > $O
for km in "4 2" "10 4"; do
  set -- $km; k=$1; m=$2; er="1,$k"
  for L in 65536 262144 1048576 4194304 16777216 67108864 268435456; do
    for th in 1 16; do
      echo "{\"impl\": \"cpu_port\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      timeout -k 10 30 tests/perf/cpu_port_native $k $m $L $th 0.6 >> $O || exit 1
    done
    for th in 1 8; do
      echo "{\"impl\": \"gpu_staged\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native $k $m $L $th 0.6 $er >> $O || exit 1
      echo "{\"impl\": \"gpu_pinned\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native $k $m $L $th 0.6 $er >> $O || exit 1
    done
  done
done
echo ok
}

# Download-side launches on the planar layout, rule against rs_plan_tune: nothing erased
# (Verify only, read-only), one data shard lost (one written row + compared rows), two lost,
# and one parity lost (tools/ceiling_sweep.py, in place). Usage: bash tools/jobs.sh decode_rule_sweep <tag>
job_decode_rule_sweep() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-decrule}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "4 2" "6 3" "8 4" "10 4" "12 4" "16 4" "10 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,none,planar" --shape "$k,$m,$S,$B,1,planar" --shape "$k,$m,$S,$B,0+1,planar" --shape "$k,$m,$S,$B,$k,planar")
  done
done
timeout -k 10 1100 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo "decode sweep ok"
}

# CallFS server default profile RS(4,2) (config/loader.go:301-304) end to end through the
# C ABI: pageable (staged) and rs_host_alloc (zero-copy) buffers, 1 and 8 request
# threads, decode erasing one data and one parity shard; CPU port beside it.
# Output: gpurun_out/e2e_rs4_2.jsonl. Usage: bash tools/jobs.sh default_profile_e2e
job_default_profile_e2e() {
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/e2e_rs4_2.jsonl; rm -f $O
for L in 1048576 16777216 67108864 268435456; do
  for th in 1 8; do
    echo "{\"mode\": \"staged\", \"threads\": $th}" >> $O
    CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 4 2 $L $th 1.0 1,4 >> $O || exit 1
    echo "{\"mode\": \"pinned\", \"threads\": $th}" >> $O
    CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 4 2 $L $th 1.0 1,4 >> $O || exit 1
  done
  for th in 1 16; do timeout -k 10 30 tests/perf/cpu_port_native 4 2 $L $th 1.0 >> $O || exit 1; done
done
echo ok
}

# LDS-DMA ring (rs_apply.hpp Policy::DMA, A/B build): bit-exact through the every-order test
# on the A/B library, then against the rule and the triple forms on R 5..8 and R <= 4 shapes
# (tools/order_ab.py, planar layout). Usage: bash tools/jobs.sh dma_probe <tag>
job_dma_probe() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-dma}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
# the A/B build is not pushed: built here on demand (build/ab/, tools/callfs_rs_ab.h)
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
export CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k every_offered > "$O/pytest_ab.log" 2>&1 || exit $?
echo "ab tests ok"
A=()
for s in 10,8,6710887,32 8,8,8388608,32 8,8,2097152,128 10,8,1677722,128 32,8,2097152,64 \
         16,8,1048576,256 10,4,1048576,256 10,4,6710887,45 8,8,131072,1024; do
  A+=(--shape "$s,-,planar")
done
timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 \
  --orders consecutive,g2,x32,tri,tri-g2,tri-x32,tri-q8,dma,dma-g2,dma-q8,dma-x32 "${A[@]}" \
  > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
}

# G8 (8 stripes interleaved) on long shards: the write-pattern probe (tools/write_pattern.hip)
# found it the best write order for 4 and 8 rows at every shard size; the ring of three in G8
# against the rule and the tuner's forms, and the read / write ceilings in G8.
# Usage: bash tools/jobs.sh g8_probe <tag>
job_g8_probe() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-g8}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for s in 10,4,6710887,256,- 10,4,6710887,256,0+1+2+3 10,8,6710887,64,- 8,8,8388608,64,- \
         10,4,8388608,64,- 10,4,1048576,256,- 16,4,4194304,128,- 10,4,16777216,32,-; do
  A+=(--shape "$s,planar")
done
timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 \
  --orders consecutive,g2,g8,q8,x32,tri,tri-g2,tri-q8,tri-x32 "${A[@]}" > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
timeout -k 10 300 python3 -u tools/ceiling_orders.py --orders consecutive,g2,g8,q8,x32 \
  --shape 10,4,6710887,256,-,planar --shape 10,8,6710887,64,-,planar > "$O/ceil.jsonl" 2>&1 || exit $?
echo "ceil ok"
}

# Full GPU pass: gpu tests, default bench, rocprofv3 passes. Usage: bash tools/jobs.sh gpu_round <tag>
job_gpu_round() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-r01}"
cd "$R"; mkdir -p "gpurun_out/$TAG"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > "gpurun_out/$TAG/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 "gpurun_out/$TAG/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/$TAG/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 "gpurun_out/$TAG/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "gpurun_out/$TAG/bench.log" 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 "gpurun_out/$TAG/bench.log"; [ $rc -eq 0 ] || exit $rc
bash "$JOBS" profile "$TAG"
}

# GPU test suite only. Usage: bash tools/jobs.sh gpu_tests <tag> [pytest -k expr] [test path]
job_gpu_tests() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-t}"; mkdir -p "$R/gpurun_out/$TAG"; cd "$R"
K=()
[ -n "$2" ] && K=(-k "$2")
P="${3:-tests}"
timeout -k 10 900 python3 -u -m pytest "$P" -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread --durations 15 "${K[@]}" > "gpurun_out/$TAG/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 "gpurun_out/$TAG/pytest_gpu.log"; exit $rc
}

# Row n1 (north_star: the end-to-end rate with pinned H2D/D2H) on the current build:
# configs[4] -- RS(16,4) encode + reconstruct {0,5,16,19} + verify + join, 4 KiB - 64 MiB
# objects, 1 and 8 request threads -- through the shim's three host paths (staged pageable
# buffers, rs_host_alloc buffers, and the BodyBuffer / DecodePinned sequence of
# tests/native/cgo_drive.c), then the CPU/GPU crossover for the shim's GPU_MIN_BYTES default
# (RS(4,2) and RS(10,4), CPU port at 1 and 16 threads). Usage: bash tools/jobs.sh n1_r06 <tag>
job_n1_r06() {
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-n1}"; mkdir -p "$OUT"
O=$OUT/cfg4_e2e.jsonl; : > $O
for L in 4096 65536 1048576 4194304 16777216 67108864; do
  for th in 1 8; do
    for mode in staged pinned body; do
      echo "{\"mode\": \"$mode\", \"threads\": $th}" >> $O
      case $mode in
        staged) env CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 16 4 $L $th 0.8 0,5,16,19 >> $O || exit 1 ;;
        pinned) env CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native 16 4 $L $th 0.8 0,5,16,19 >> $O || exit 1 ;;
        body) env CALLFS_E2E_BODY=1 timeout -k 10 60 tools/e2e_native 16 4 $L $th 0.8 0,5,16,19 >> $O || exit 1 ;;
      esac
    done
  done
done
echo "cfg4 ok"
O=$OUT/crossover.jsonl; : > $O
for km in "4 2" "10 4"; do
  set -- $km; k=$1; m=$2; er="1,$k"
  for L in 1048576 4194304 16777216 67108864 268435456; do
    for th in 1 16; do
      echo "{\"impl\": \"cpu_port\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      timeout -k 10 30 tests/perf/cpu_port_native $k $m $L $th 0.6 >> $O || exit 1
    done
    for th in 1 8; do
      echo "{\"impl\": \"gpu_staged\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      CALLFS_E2E_ENCODER=1 timeout -k 10 60 tools/e2e_native $k $m $L $th 0.6 $er >> $O || exit 1
      echo "{\"impl\": \"gpu_body\", \"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th}" >> $O
      CALLFS_E2E_BODY=1 timeout -k 10 60 tools/e2e_native $k $m $L $th 0.6 $er >> $O || exit 1
    done
  done
done
echo "crossover ok"
}

# Is the kernel's compute exposed? The production launch against its no-lookup form (same
# loads, stores, grid, order; A/B build) and the read / write ceilings, on R 5..8 and wide
# shapes and on the bench shape (tools/ceiling_sweep.py). Usage: bash tools/jobs.sh nolookup_probe <tag>
job_nolookup_probe() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-nolookup}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
# the A/B build is not pushed: built here on demand (build/ab/, tools/callfs_rs_ab.h)
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
export CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so"
A=()
for s in 10,4,1048576,256 10,4,6710887,64 10,8,6710887,32 8,8,8388608,32 32,8,2097152,64 \
         16,8,1048576,256 10,16,1048576,128 20,16,1048576,96 32,16,1048576,64; do
  A+=(--shape "$s,-,planar")
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --rounds 2 "${A[@]}" > "$O/sweep.jsonl" 2>&1 || exit $?
echo "nolookup ok"
}

# Shard-pitch study for BASELINE configs[1]/[2] (RS(10,4), 64 MiB objects, S = 6,710,887)
# in the planar layout: pitch = round_up(S, 2^p) for p = 8..23 and 256-B pitch + 4/8/64 KiB,
# encode and the 4-erasure decode, rule and tuned plus the read / write ceilings
# (tools/ceiling_sweep.py, layout 'planar:P'). Usage: bash tools/jobs.sh pitch_sweep <tag> [k m S]
job_pitch_sweep() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-pitch}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
k=${2:-10}; m=${3:-4}; S=${4:-6710887}
P=$(python3 - "$S" <<'EOF'
import sys
S = int(sys.argv[1])
up = lambda a: -(-S // a) * a
ps = []
for p in list(range(8, 24)):
    q = up(1 << p)
    if q not in ps:
        ps.append(q)
for extra in (4096, 8192, 65536):
    q = up(256) + extra
    if q not in ps:
        ps.append(q)
print(" ".join(str(x) for x in ps))
EOF
) || exit 1
echo "pitches: $P"
B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
A=()
for p in $P; do
  A+=(--shape "$k,$m,$S,$B,-,planar:$p" --shape "$k,$m,$S,$B,0+1+2+3,planar:$p")
done
timeout -k 10 1000 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned,read,write "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo "sweep ok"
}

# Counter table of the bit-sliced kernels against the nibble-table kernel on wide shapes
# (what binds each): per (shape, form) a kernel trace and PMC passes of tools/plan_run.py.
# Product library. Usage: bash tools/jobs.sh pmc_bs <tag> <shape> <order> [<order> ...]
job_pmc_bs() {
R="$GRAFT_REPO_ROOT"; TAG="$1"; SH="$2"; shift 2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
[ -f "$OUT/../avail.txt" ] || timeout -k 10 120 rocprofv3 --list-avail > "$OUT/../avail.txt" 2>&1 || true
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
PB="GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
IC=$(grep -o "SQC_ICACHE_[A-Z_]*" "$OUT/../avail.txt" | sort -u | grep -E "^SQC_ICACHE_(MISSES|HITS|REQ)$" | head -3 | tr '\n' ' ')
for o in "$@"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$o" -o run -- \
    python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 30 > "$OUT/trace_$o.log" 2>&1 || { echo "trace $o rc=$?"; exit 1; }
  for p in A B C; do
    eval "C=\$P$p"
    [ "$p" = C ] && C="$IC"
    [ -z "$C" ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${o}_$p" -o pmc -- \
      python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 8 > "$OUT/pmc_${o}_$p.log" 2>&1
    rc=$?
    case $rc in 0) ;; *) echo "pass $p of $o rc=$rc: stop"; tail -3 "$OUT/pmc_${o}_$p.log"; exit $rc ;; esac
  done
  echo "$o ok"
done
}

# Counter table of kernel forms on one shape (what binds R 5..8): per form a kernel trace
# (time) and two PMC passes (tools/plan_run.py under rocprofv3), A/B build of the library.
# Usage: bash tools/jobs.sh pmc_forms <tag> <shape> <order> [<order> ...]
job_pmc_forms() {
R="$GRAFT_REPO_ROOT"; TAG="$1"; SH="$2"; shift 2; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
# the A/B build is not pushed: built here on demand (build/ab/, tools/callfs_rs_ab.h)
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
export CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so"
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for o in "$@"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$o" -o run -- \
    python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 30 > "$OUT/trace_$o.log" 2>&1 || { echo "trace $o rc=$?"; exit 1; }
  for p in A B; do
    eval "C=\$P$p"
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${o}_$p" -o pmc -- \
      python3 "$R/tools/plan_run.py" --shape "$SH" --order "$o" --launches 8 > "$OUT/pmc_${o}_$p.log" 2>&1
    rc=$?
    case $rc in 0) ;; *) echo "pass $p of $o rc=$rc: stop"; tail -3 "$OUT/pmc_${o}_$p.log"; exit $rc ;; esac
  done
  echo "$o ok"
done
}

# rocprofv3 passes for the bench workload. Usage: bash tools/jobs.sh profile <tag> [bench args]
# 1) --kernel-trace --stats  2) --pmc FETCH_SIZE  3) --pmc WRITE_SIZE (separate passes)
job_profile() {
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
}

# configs[1]/[2] shape in the layouts upstream produces: bench.py at S = 6,710,887 with the
# io.ReadAll Split layout (decode into fresh buffers, as Reconstruct allocates them, and in
# place) and the planar layout; plus the bench shape. Usage: bash tools/jobs.sh readall_bench <tag>
job_readall_bench() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-readall}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
run() { timeout -k 10 300 python3 -u bench.py --steps 20 --cpu-seconds 0 --layout-ab 0 "$@"; }
run --shard-bytes 6710887 --split-layout readall > "$O/readall_fresh.log" 2>&1 || exit $?
run --shard-bytes 6710887 --split-layout readall --decode-into inplace > "$O/readall_inplace.log" 2>&1 || exit $?
run --shard-bytes 6710887 > "$O/planar_cfg12.log" 2>&1 || exit $?
run > "$O/planar_bench.log" 2>&1 || exit $?
echo "benches ok"
}

# Round 5's 40 seeded io.ReadAll one-shard decodes (profiles/r05/tiles/random_readall_dec1_*;
# shapes in tools/readall_dec1_shapes.txt), rule against tuner, decode into fresh buffers, on
# the current build. Usage: bash tools/jobs.sh readall_dec1_r06 <tag>
job_readall_dec1_r06() {
cd "$GRAFT_REPO_ROOT"; O="gpurun_out/${1:-readall_dec1}"; mkdir -p "$O"
A=(); while read -r s; do [ -n "$s" ] && A+=(--shape "$s"); done < tools/readall_dec1_shapes.txt
timeout -k 10 1000 python3 -u tools/ceiling_sweep.py --tune 1 --fresh 1 --only prod,tuned --rounds 2 "${A[@]}" > "$O/sweep.jsonl" 2> "$O/sweep.err" || exit $?
echo ok
}

# The profile sweep's 33 cells in the layout CallFS produces (upstream Split of an io.ReadAll
# body: data shards at pitch S in the body, parity in 64-B AllocAligned buffers), encode and a
# two-data-shard decode (in place; FRESH=1: into fresh buffers, as upstream Reconstruct
# allocates them), rule against rs_plan_tune (tools/ceiling_sweep.py).
# Usage: [FRESH=1] bash tools/jobs.sh readall_rule_sweep <tag>
job_readall_rule_sweep() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-readall_rule}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,readall" --shape "$k,$m,$S,$B,0+1,readall")
  done
done
timeout -k 10 1300 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned --fresh "${FRESH:-0}" "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo "readall sweep ok"
}

# N > 1 launch rehearsal on a 1-GPU box (ranks share the device, LOCAL_RANK % device_count):
# the driver's torchrun line at N = 4 (weak, default workload) and the configs[3] column
# split (1 GiB objects, strong) at N = 1 and 4. Usage: bash tools/jobs.sh rehearse_ranks <tag>
job_rehearse_ranks() {
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
}

# Round-end evidence in one call: GPU tests, smoke, bench line, rocprofv3 passes (gpu_round.sh),
# one pass of the planar rule sweep, and the write-pattern probe. Usage: bash tools/jobs.sh round_final <tag>
job_round_final() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-final}"; cd "$R"
bash "$JOBS" gpu_round "$TAG" || exit $?
A=()
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,planar")
  done
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "gpurun_out/$TAG/rule_sweep.jsonl" 2>&1 || exit $?
echo "rule sweep ok"
timeout -k 10 300 tools/write_pattern 6 > "gpurun_out/$TAG/write_pattern_bs.csv" 2>&1 || exit $?
echo "write pattern ok"
# the double-buffered triples with 4 / 8 stripes interleaved (A/B build): bit-exact, then
# against the rule's tri-G2 on the bench shape and its neighbours
timeout -k 10 900 python3 callfs_amd/build.py --ab > /dev/null || exit $?
CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so" timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py -k every_offered > "gpurun_out/$TAG/pytest_ab.log" 2>&1 || exit $?
echo "ab tests ok"
A=()
for s in 10,4,1048576,256 10,4,1048576,512 16,4,1048576,256 8,4,2097152,128 12,4,1398102,128 10,4,104858,1024 6,3,174763,2048; do
  A+=(--shape "$s,-,planar")
done
CALLFS_RS_LIB="$R/build/ab/libcallfs_rs_ab.so" timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 \
  --orders tri-g2,tridb-g4,tridb-g8,tri-x32 "${A[@]}" > "gpurun_out/$TAG/tridb_g.jsonl" 2>&1 || exit $?
echo "tridb-g ok"
}

# The profile sweep's 33 cells (11 RS profiles x 1, 16, 64 MiB objects, ~4 GiB batches) in
# the planar layout (the bench layout), production rule against rs_plan_tune, two passes
# (tools/ceiling_sweep.py): the data the tile-order rule is fitted to (tile_order.hpp).
# Usage: [PASSES=n] bash tools/jobs.sh rule_sweep <tag> [extra ceiling_sweep args]
job_rule_sweep() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-rule}"; shift; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "4 2" "3 2" "6 3" "8 4" "10 4" "12 4" "16 4" "8 8" "10 8" "20 4" "32 8"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,planar")
  done
done
for pass in $(seq 1 "${PASSES:-2}"); do
  timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
    > "$O/sweep_$pass.jsonl" 2>&1 || exit $?
  echo "pass $pass ok"
done
}

# Launch-slice size (CALLFS_RS_MAX_TILES_PER_LAUNCH, rs_kernels.hip slice_tiles) on the
# configs[1] shape (RS(10,4), S = 6,710,887, planar, 256 stripes = 24 GB per launch) and on
# the bench shape, rule and tuned plus the read / write ceilings; one process per setting.
# Usage: bash tools/jobs.sh slice_probe <tag>
job_slice_probe() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-slice}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
for T in 0 4096 8192 16384 65536 1000000000; do
  if [ $T = 0 ]; then unset CALLFS_RS_MAX_TILES_PER_LAUNCH; else export CALLFS_RS_MAX_TILES_PER_LAUNCH=$T; fi
  timeout -k 10 300 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned,read,write \
    --shape 10,4,6710887,256,-,planar --shape 10,4,6710887,256,0+1+2+3,planar \
    --shape 10,4,1048576,256,-,planar > "$O/slice_$T.jsonl" 2>&1 || exit $?
  echo "slice $T ok"
done
}

# One-dispatch small path vs the staged path (CALLFS_RS_SMALL_MAX_BYTES=0), RS(16,4)
# encoder path + decode {0,5,16,19} and RS(4,2) {1,4}, 1 and 8 threads, host buffers.
# Usage: bash tools/jobs.sh small_path_sweep <tag>
job_small_path_sweep() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-smallpath}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; O="$OUT/sweep.jsonl"
export CALLFS_E2E_ENCODER=1
for prof in "16 4 0,5,16,19" "4 2 1,4"; do
  set -- $prof
  for L in ${SIZES:-4096 16384 65536 262144 1048576}; do
    for t in 1 8; do
      for mode in staged small; do
        lim=$([ $mode = staged ] && echo 0 || echo ${SMALL_LIM:-67108864})
        echo "{\"mode\": \"$mode\", \"small_max\": $lim}" >> $O
        CALLFS_RS_SMALL_MAX_BYTES=$lim timeout -k 10 60 "$R/tools/e2e_native" $1 $2 $L $t 0.6 $3 >> $O || exit 1
      done
    done
  done
done
echo ok
}

# Does the best form at long shards depend on the batch size? RS(10,4) at 6.7 MB and 8 MiB
# shards with 45..256 stripes, the ring (consecutive) against the triple forms (tools/order_ab.py).
# Usage: bash tools/jobs.sh stripes_probe <tag>
job_stripes_probe() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-stripes}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for s in 10,4,6710887,45 10,4,6710887,128 10,4,6710887,256 10,4,8388608,36 10,4,8388608,128 \
         10,4,8388608,200 12,4,5592406,54 12,4,5592406,256; do
  A+=(--shape "$s,-,planar")
done
timeout -k 10 600 python3 -u tools/order_ab.py --rounds 3 --orders consecutive,x32,tri-q8,tri-x32 "${A[@]}" \
  > "$O/orders.jsonl" 2>&1 || exit $?
echo "orders ok"
}

# Wide and many-input profiles (the bit-sliced kernels' launches) at 1, 16 and 64 MiB
# objects, ~4 GiB batches, planar: production rule against rs_plan_tune (which also times
# the nibble-table forms). Usage: bash tools/jobs.sh wide_sweep_r06 <tag>
job_wide_sweep_r06() {
R="$GRAFT_REPO_ROOT"; TAG="${1:-wide}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
A=()
for km in "10 16" "20 16" "32 16" "16 8" "24 12" "20 9"; do
  set -- $km; k=$1; m=$2
  for L in 1048576 16777216 67108864; do
    S=$(( (L + k - 1) / k )); B=$(( (4 << 30) / (S * (k + m)) )); [ $B -lt 1 ] && B=1
    A+=(--shape "$k,$m,$S,$B,-,planar")
  done
done
timeout -k 10 900 python3 -u tools/ceiling_sweep.py --tune 1 --rounds 2 --only prod,tuned "${A[@]}" \
  > "$O/sweep.jsonl" 2>&1 || exit $?
echo ok
}

# Zero-copy threshold (CALLFS_RS_ZERO_COPY_MIN_BYTES, rs_capi.cpp zc_min) on the current
# build: rs_host_alloc buffers through the zero-copy launch (threshold 1 B) against the
# one-dispatch small path / staged pipeline (threshold 1 GiB), encode + decode, 1 and 8
# request threads. Output: gpurun_out/<tag>/zc.jsonl. Usage: bash tools/jobs.sh zc_threshold <tag>
job_zc_threshold() {
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/${1:-zc_threshold}"; mkdir -p "$OUT"; O=$OUT/zc.jsonl; : > $O
for km in "16 4" "10 4" "4 2"; do
  set -- $km; k=$1; m=$2
  for L in 131072 262144 393216 524288 786432 1048576 1572864; do
    for th in 1 8; do
      for zc in 1 1073741824; do
        echo "{\"k\": $k, \"m\": $m, \"L\": $L, \"threads\": $th, \"zc_min\": $zc}" >> $O
        CALLFS_RS_ZERO_COPY_MIN_BYTES=$zc CALLFS_E2E_PINNED=1 CALLFS_E2E_ENCODER=1 \
          timeout -k 10 60 tools/e2e_native $k $m $L $th 0.5 0,$k >> $O || exit 1
      done
    done
  done
done
echo ok
}

if [ $# -lt 1 ] || ! declare -F "job_$1" > /dev/null; then
  echo "usage: bash tools/jobs.sh <job> [args]" >&2
  declare -F | sed -n 's/^declare -f job_/  /p' >&2
  exit 2
fi
j=$1; shift
"job_$j" "$@"
