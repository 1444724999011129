#!/bin/bash
# kernel-efficiency round: numerics of the touched kernels, the loopback per-rank TeraSort and the
# k-means job, then kernel statistics of both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail 10 -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5k_tests.log 2>&1 || { tail -30 gpurun_out/r5k_tests.log; exit 1; }
tail -1 gpurun_out/r5k_tests.log
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r5k_lb8.log 2>&1 || { tail -20 gpurun_out/r5k_lb8.log; exit 1; }
tail -1 gpurun_out/r5k_lb8.log | cut -c1-600
timeout -k 10 300 python -u benchmarks/kmeans.py > gpurun_out/r5k_km.log 2>&1 || { tail -20 gpurun_out/r5k_km.log; exit 1; }
tail -3 gpurun_out/r5k_km.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5k_lb -o run --output-format csv -- \
  python3 bench.py --loopback-ranks 8 --steps 2 --warmup 1 > gpurun_out/r5k_lb8_prof.log 2>&1 || { tail -20 gpurun_out/r5k_lb8_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5k_km -o run --output-format csv -- \
  python3 benchmarks/kmeans.py --iters 3 > gpurun_out/r5k_km_prof.log 2>&1 || { tail -20 gpurun_out/r5k_km_prof.log; exit 1; }
find gpurun_out/prof_r5k_lb gpurun_out/prof_r5k_km -name '*kernel_stats.csv' | head
