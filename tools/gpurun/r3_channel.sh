#!/bin/bash
# Channel kernels + device exchange: kernel numerics, executor tests, multi-rank sweeps on one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_channel.py tests/test_gpu_executor.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_channel.log 2>&1 || { tail -60 gpurun_out/r3_channel.log; exit 1; }
tail -3 gpurun_out/r3_channel.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r3_multirank.log 2>&1 || { tail -80 gpurun_out/r3_multirank.log; exit 1; }
tail -12 gpurun_out/r3_multirank.log
