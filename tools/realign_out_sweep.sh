# Split-layout (odd S, pitch = S) shapes: the plain kernel (unaligned loads and stores),
# realigned loads (REALIGN 1) and realigned loads + parity stores (REALIGN 2), with the
# unaligned no-lookup ceiling. Usage: bash tools/realign_out_sweep.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-ro}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_PROBE63=1 KB_KEEP="realign consec|realign out|plain consec|nomath consec"
run() {  # name k m S B
  timeout -k 10 200 "$R/tools/kbench" $2 $3 $4 $5 7 10 1 > "$OUT/$1.log" 2>&1 || exit $?
  grep -vE "^RS|variant" "$OUT/$1.log" | sed "s/^/$1 /"
}
run split_4_2_1m 4 2 1048577 512
run split_6_3_1m 6 3 1048577 256
run split_5_3_1m 5 3 1048577 256
run split_16_4_256k 16 4 262145 256
run split_10_4_1m 10 4 1048577 256
run split_12_4_64m 12 4 5592406 64
run split_10_4_even 10 4 1048578 256
run split_10_8_1m 10 8 1048577 256
