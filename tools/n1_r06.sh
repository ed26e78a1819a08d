# Row n1 (north_star: the end-to-end rate with pinned H2D/D2H) on the current build:
# configs[4] -- RS(16,4) encode + reconstruct {0,5,16,19} + verify + join, 4 KiB - 64 MiB
# objects, 1 and 8 request threads -- through the shim's three host paths (staged pageable
# buffers, rs_host_alloc buffers, and the BodyBuffer / DecodePinned sequence of
# tests/native/cgo_drive.c), then the CPU/GPU crossover for the shim's GPU_MIN_BYTES default
# (RS(4,2) and RS(10,4), CPU port at 1 and 16 threads). Usage: bash tools/n1_r06.sh <tag>
set -o pipefail
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
