#!/bin/bash
# GPU check (gpurun): the new device-op tests first, then the whole GPU suite, the op
# microbenchmarks and the headline bench.  Every GPU step has its own time limit; the script
# stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_ops.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_new.log 2>&1 || { tail -60 gpurun_out/gpu_new.log; exit 1; }
tail -3 gpurun_out/gpu_new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u tools/microbench_ops.py > gpurun_out/microbench_ops.log 2>&1 \
  || { tail -20 gpurun_out/microbench_ops.log; exit 1; }
cat gpurun_out/microbench_ops.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
