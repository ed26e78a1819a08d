# Is the realigning kernel's 63-vector wave tiling (1,008-B wave windows) what costs it
# ~5 points on aligned shards? Plain kernel with 63-vector waves vs 64-vector waves with
# lane 63 idle, aligned and Split-layout shards. Usage: bash tools/wave_tiling_probe.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-wtp}"
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
export KB_PROBE63=1 KB_KEEP="probe 6|realign consec|realign out|plain consec|nomath consec"
run() {  # name k m S B palign
  timeout -k 10 200 "$R/tools/kbench" $2 $3 $4 $5 7 10 $6 > "$OUT/$1.log" 2>&1 || exit $?
  grep -vE "^RS|variant" "$OUT/$1.log" | sed "s/^/$1 /"
}
run aligned_10_4_1m 10 4 1048576 256 256
run split_10_4_64m 10 4 6710887 64 1
run aligned_10_4_64m 10 4 6710887 64 256
run split_10_8_1m 10 8 1048577 256 1
