#!/bin/bash
# Round-3 k-means: numerics (split planes + f32 path), microbench at 125M x 128, the BASELINE
# k-means job, and a kernel-trace profile of the job.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_hipgraph.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/km_tests.log 2>&1 || { tail -40 gpurun_out/km_tests.log; exit 1; }
tail -2 gpurun_out/km_tests.log
timeout -k 10 300 python -u tools/microbench_kmeans.py 125e6 64 > gpurun_out/km_micro.log 2>&1 || { tail -20 gpurun_out/km_micro.log; exit 1; }
cat gpurun_out/km_micro.log
timeout -k 10 300 python -u benchmarks/kmeans.py > gpurun_out/km_bench.log 2>&1 || { tail -30 gpurun_out/km_bench.log; exit 1; }
grep metric gpurun_out/km_bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/km_prof -o km --output-format csv -- python3 benchmarks/kmeans.py --iters 3 \
  > gpurun_out/km_prof.log 2>&1 || { tail -20 gpurun_out/km_prof.log; exit 1; }
find gpurun_out/km_prof -name "*kernel_stats.csv" | head -3
