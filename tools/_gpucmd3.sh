#!/bin/bash
# re-check the reduce kernel (adjacent-slot load reuse), measure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_ops.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/gpu_t3.log 2>&1 || { tail -40 gpurun_out/gpu_t3.log; exit 1; }
tail -2 gpurun_out/gpu_t3.log
timeout -k 10 300 python -u tools/microbench_ops.py > gpurun_out/microbench_ops.log 2>&1 \
  || { tail -20 gpurun_out/microbench_ops.log; exit 1; }
head -6 gpurun_out/microbench_ops.log
