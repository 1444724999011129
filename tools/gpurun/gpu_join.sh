#!/bin/bash
# grace hash join: kernel tests, then the 2 x 100 GB benchmark (HBM-resident default and a forced
# HBM budget that spills to pinned host DRAM).  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_grace.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/grace_tests.log 2>&1 || { tail -40 gpurun_out/grace_tests.log; exit 1; }
tail -1 gpurun_out/grace_tests.log
cd benchmarks || exit 1
timeout -k 10 300 python -u join.py --steps 3 --warmup 1 > ../gpurun_out/join.log 2>&1 || { tail -20 ../gpurun_out/join.log; exit 1; }
tail -1 ../gpurun_out/join.log
if [ "$1" = "spill" ]; then
  timeout -k 10 400 python -u join.py --steps 2 --warmup 1 --hbm-budget-gb 130 > ../gpurun_out/join_spill.log 2>&1 \
    || { tail -20 ../gpurun_out/join_spill.log; exit 1; }
  tail -1 ../gpurun_out/join_spill.log
fi
