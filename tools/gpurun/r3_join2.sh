#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py tests/test_gpu_grace.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_join_tests.log 2>&1 || { tail -60 gpurun_out/r3_join_tests.log; exit 1; }
tail -2 gpurun_out/r3_join_tests.log
timeout -k 10 400 python -u benchmarks/join.py --steps 3 > gpurun_out/r3_join_hbm.log 2>&1 || { tail -30 gpurun_out/r3_join_hbm.log; exit 1; }
grep '"metric"' gpurun_out/r3_join_hbm.log | cut -c1-1500
timeout -k 10 500 python -u benchmarks/join.py --hbm-budget-gb 30 > gpurun_out/r3_join_spill.log 2>&1 || { tail -30 gpurun_out/r3_join_spill.log; exit 1; }
grep '"metric"' gpurun_out/r3_join_spill.log | cut -c1-1500
timeout -k 10 500 python -u benchmarks/join.py --hbm-budget-gb 130 > gpurun_out/r3_join_130.log 2>&1 || { tail -30 gpurun_out/r3_join_130.log; exit 1; }
grep '"metric"' gpurun_out/r3_join_130.log | cut -c1-1500
