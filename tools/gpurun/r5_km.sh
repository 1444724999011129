#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_tsmerge.py tests/test_gpu_kmeans.py tests/test_gpu_fine_rows.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_tm_tests.log 2>&1 || { tail -30 gpurun_out/r5_tm_tests.log; exit 1; }
tail -1 gpurun_out/r5_tm_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r5_km_ab -o run --output-format csv -- \
  python3 tools/micro/km_depth_ab.py > gpurun_out/r5_km_ab.log 2>&1 || { tail -20 gpurun_out/r5_km_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_km_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_tm -o run --output-format csv -- \
  python3 bench.py --loopback-ranks 8 --steps 2 --warmup 1 > gpurun_out/r5_tm_lb8.log 2>&1 || { tail -20 gpurun_out/r5_tm_lb8.log; exit 1; }
tail -1 gpurun_out/r5_tm_lb8.log | cut -c1-200
grep -h "tile_merge\|pack_rows" gpurun_out/prof_r5_tm/run_kernel_stats.csv | cut -c1-200
