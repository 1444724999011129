#!/bin/bash
# packed-row vector loads in the segmented reduction: tests, GroupBy benchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_ops.py tests/test_gpu_executor.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/gpu_t3.log 2>&1 || { tail -40 gpurun_out/gpu_t3.log; exit 1; }
tail -2 gpurun_out/gpu_t3.log
cd benchmarks || exit 1
timeout -k 10 300 python -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/gb.log 2>&1 || { tail -20 ../gpurun_out/gb.log; exit 1; }
tail -1 ../gpurun_out/gb.log
