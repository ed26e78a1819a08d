set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/shift
export KB_SHIFT=1 KB_KEEP="lds shift|lds prod-policy|lds bs512 (prod"
for cfg in "10 4 1048576 256" "4 2 1048576 512" "10 8 1048576 256" "16 4 4194304 64"; do
  timeout -k 10 120 tools/kbench $cfg 7 10 > "gpurun_out/shift/kb_${cfg// /_}.log" 2>&1 || exit $?
done
echo ok
