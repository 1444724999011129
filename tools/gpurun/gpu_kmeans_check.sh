#!/bin/bash
# k-means check for gpurun: numerics tests, the BASELINE k-means config, and a kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/km_tests.log 2>&1 || { tail -40 gpurun_out/km_tests.log; exit 1; }
tail -2 gpurun_out/km_tests.log
timeout -k 10 300 python -u benchmarks/kmeans.py > gpurun_out/km_bench.log 2>&1 || { tail -30 gpurun_out/km_bench.log; exit 1; }
tail -4 gpurun_out/km_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/km_prof -o km -- python3 benchmarks/kmeans.py --iters 3 \
  > gpurun_out/km_prof.log 2>&1 || { tail -20 gpurun_out/km_prof.log; exit 1; }
find gpurun_out/km_prof -name "*kernel_stats.csv" | head -3
