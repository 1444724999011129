#!/bin/bash
# 128-byte-pitch TeraSort input: its tests, the sort/executor suites, then the headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pitch128.py tests/test_gpu_compact_sort.py tests/test_gpu_executor.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pitch_tests.log 2>&1 || { tail -40 gpurun_out/pitch_tests.log; exit 1; }
tail -2 gpurun_out/pitch_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/pitch_bench.log 2>&1 || { tail -30 gpurun_out/pitch_bench.log; exit 1; }
grep '"metric"' gpurun_out/pitch_bench.log | cut -c1-300
grep "HBM free\|executor" gpurun_out/pitch_bench.log | cut -c1-600
