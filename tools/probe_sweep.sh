# Does a read probe rank tile orders like the kernel? KB_ORD kernel variants + KB_PROBE
# read probes per shape. Usage: bash tools/probe_sweep.sh <tag> "k m S B" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/$1"; shift; mkdir -p "$OUT"
for shape in "$@"; do
  set -- $shape
  KB_ORD=1 KB_PROBE=1 KB_KEEP="lds ord consec|lds ord g8|lds ord g2|lds ord q8|lds ord q16|lds ord q64|probe" timeout -k 10 120 tools/kbench $1 $2 $3 $4 5 10 > "$OUT/kb_$1_$2_$3_$4.log" 2>&1 || exit $?
  echo "== $shape"
done
