set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-pd}"; mkdir -p "$OUT"
export KB_SDWA=1 KB_PROD2=1
for keep in "sdwa|perm|prod dispatch (2nd)" "sdwa|perm|prod dispatch (2nd)|nomath g2"; do
  export KB_KEEP="$keep"
  for sh in 10,4 10,16; do k=${sh%,*}; m=${sh#*,}
    timeout -k 10 200 "$R/tools/kbench" $k $m 1048576 256 7 10 > "$OUT/kb_${k}_${m}_${#keep}.log" 2>&1 || exit $?
    grep -vE "^RS|variant" "$OUT/kb_${k}_${m}_${#keep}.log" | sed "s/^/RS($k,$m) keep${#keep} /"
  done
done
