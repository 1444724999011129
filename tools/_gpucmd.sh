#!/bin/bash
# GPU check (gpurun): the whole GPU suite, smoke(), the headline bench and the secondary BASELINE
# benchmarks.  Every GPU step has its own time limit; the script stops at the first failure.
# Pass "secondary" to run only the secondary benchmarks.
set -o pipefail
mkdir -p gpurun_out
if [ "$1" != "secondary" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
  timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
cd benchmarks || exit 1
timeout -k 10 300 python -u groupby.py > ../gpurun_out/gb.log 2>&1 || { tail -20 ../gpurun_out/gb.log; exit 1; }
tail -1 ../gpurun_out/gb.log
timeout -k 10 300 python -u kmeans.py > ../gpurun_out/km.log 2>&1 || { tail -20 ../gpurun_out/km.log; exit 1; }
tail -1 ../gpurun_out/km.log
timeout -k 10 400 python -u join.py > ../gpurun_out/join.log 2>&1 || { tail -20 ../gpurun_out/join.log; exit 1; }
tail -1 ../gpurun_out/join.log
