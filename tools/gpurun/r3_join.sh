#!/bin/bash
# Fused grace join through the API: GPU tests, then the BASELINE join config (in HBM, then a budget
# that forces spill), and the multi-rank sweep with the fused join on 2 ranks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py tests/test_gpu_channel.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_join_tests.log 2>&1 || { tail -60 gpurun_out/r3_join_tests.log; exit 1; }
tail -2 gpurun_out/r3_join_tests.log
timeout -k 10 400 python -u benchmarks/join.py > gpurun_out/r3_join_hbm.log 2>&1 || { tail -30 gpurun_out/r3_join_hbm.log; exit 1; }
grep '"metric"' gpurun_out/r3_join_hbm.log | cut -c1-1500
timeout -k 10 500 python -u benchmarks/join.py --hbm-budget-gb 30 > gpurun_out/r3_join_spill.log 2>&1 || { tail -30 gpurun_out/r3_join_spill.log; exit 1; }
grep '"metric"' gpurun_out/r3_join_spill.log | cut -c1-1500
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 580 --timeout-method thread -k "sweep_ranks and 2 or exchange" \
  > gpurun_out/r3_mr.log 2>&1 || { tail -40 gpurun_out/r3_mr.log; exit 1; }
tail -6 gpurun_out/r3_mr.log
