set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 500 --timeout-method thread > gpurun_out/mr.log 2>&1 || { tail -40 gpurun_out/mr.log; exit 1; }
tail -1 gpurun_out/mr.log
for it in 32 16; do
  DRYAD_SORT64_ITEMS=$it timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/b_it$it.log 2>&1 || { tail -20 gpurun_out/b_it$it.log; exit 1; }
  echo "items $it: $(tail -1 gpurun_out/b_it$it.log | cut -c1-200)"
done
