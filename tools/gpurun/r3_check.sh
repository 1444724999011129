#!/bin/bash
# Round-3 GPU check: GPU tests (one process, per-test time limit), then the headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_tests.log 2>&1 || { tail -60 gpurun_out/r3_tests.log; exit 1; }
tail -3 gpurun_out/r3_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench.log 2>&1 || { tail -30 gpurun_out/r3_bench.log; exit 1; }
grep '"metric"' gpurun_out/r3_bench.log | cut -c1-400
