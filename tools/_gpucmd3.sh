#!/bin/bash
# GroupBy representatives without the full row permutation: tests, GroupBy benchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
cd benchmarks || exit 1
timeout -k 10 300 python -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/gb.log 2>&1 || { tail -20 ../gpurun_out/gb.log; exit 1; }
tail -1 ../gpurun_out/gb.log
