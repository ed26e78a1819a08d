# Native e2e sweep: the C ABI called from native threads (like the Go server's goroutines).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/e2e
rm -f gpurun_out/e2e/native.jsonl
for thr in 1 8 32; do
  for L in 4096 65536 262144 1048576 16777216 67108864; do
    timeout -k 10 60 tools/e2e_native 16 4 $L $thr 1.0 0,5,16,19 >> gpurun_out/e2e/native.jsonl || exit 1
  done
done
for L in 10485760 67108864 1073741824; do timeout -k 10 60 tools/e2e_native 10 4 $L 1 2.0 0,1,2,3 >> gpurun_out/e2e/native.jsonl || exit 1; done
timeout -k 10 60 tools/e2e_native 10 4 67108864 8 2.0 0,1,2,3 >> gpurun_out/e2e/native.jsonl || exit 1
timeout -k 10 60 tools/e2e_native 3 2 1048576 1 2.0 1 >> gpurun_out/e2e/native.jsonl || exit 1
echo sweep done
