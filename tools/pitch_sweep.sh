# Shard-pitch study for BASELINE configs[1]/[2] (RS(10,4), 64 MiB objects, S = 6,710,887)
# in the planar layout: pitch = round_up(S, 2^p) for p = 8..23 and 256-B pitch + 4/8/64 KiB,
# encode and the 4-erasure decode, rule and tuned plus the read / write ceilings
# (tools/ceiling_sweep.py, layout 'planar:P'). Usage: bash tools/pitch_sweep.sh <tag> [k m S]
set -o pipefail
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
