#!/bin/bash
# GroupBy: raw-partial test + per-rank loopback of the 8-GPU GroupBy
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_agg.py -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r5_gb_tests.log 2>&1 || { tail -40 gpurun_out/r5_gb_tests.log; exit 1; }
tail -2 gpurun_out/r5_gb_tests.log
cd benchmarks
timeout -k 10 400 python3 -u groupby.py --loopback-ranks 8 --steps 3 --warmup 1 > ../gpurun_out/r5_gb_lb8_adaptive.log 2>&1 || { tail -20 ../gpurun_out/r5_gb_lb8_adaptive.log; exit 1; }
tail -1 ../gpurun_out/r5_gb_lb8_adaptive.log
