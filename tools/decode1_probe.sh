# One-erasure decode of RS(10,4) (1 written + 3 compared rows) as kbench sees it: the
# production dispatch, tile orders and the no-lookup ceiling with the same streams.
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG="${1:-d1}"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
run() { name=$1; shift; env "$@" timeout -k 10 200 "$R/tools/kbench" 10 4 1048576 256 5 10 > "$OUT/$name.log" 2>&1 || exit $?;
        grep -E "^(prod|lds ord|nomath)|verify_mask|MISMATCH" "$OUT/$name.log" | sed "s/^/$name /"; }
run encode KB_ORD=1 KB_KEEP="lds ord|nomath"
run erase5 KB_ORD=1 KB_KEEP="lds ord|nomath" KB_IN=0,1,2,3,4,6,7,8,9,10 KB_OUT=5,11,12,13 KB_VERIFY=0xe
run erase13 KB_ORD=1 KB_KEEP="lds ord|nomath" KB_IN=0,1,2,3,4,5,6,7,8,9 KB_OUT=13,10,11,12 KB_VERIFY=0xe
run erase5_noverify KB_ORD=1 KB_KEEP="lds ord|nomath" KB_IN=0,1,2,3,4,6,7,8,9,10 KB_OUT=5,11,12,13
