#!/bin/bash
# End-of-session GPU check: every GPU test, the headline bench, smoke(), and the secondary
# BASELINE benchmarks.  Each GPU step has its own limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
grep '"metric"' gpurun_out/final_bench.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
for b in kmeans groupby join; do
  timeout -k 10 400 python -u benchmarks/$b.py > gpurun_out/final_$b.log 2>&1 || { tail -20 gpurun_out/final_$b.log; exit 1; }
  grep '"metric"' gpurun_out/final_$b.log | cut -c1-400
done
