#!/bin/bash
# k-means assignment: centroid LDS pitch 144 (conflict-free fragment reads) and prefetch depth 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kmeans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b_km_tests.log 2>&1 || { tail -30 gpurun_out/r5b_km_tests.log; exit 1; }
tail -1 gpurun_out/r5b_km_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r5b_km_ab -o run --output-format csv -- \
  python3 tools/micro/km_depth_ab.py > gpurun_out/r5b_km_ab.log 2>&1 || { tail -20 gpurun_out/r5b_km_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5b_km_ab.log
python3 tools/micro/km_ab_trace.py gpurun_out/prof_r5b_km_ab/run_kernel_trace.csv > gpurun_out/r5b_km_ab_kernels.txt 2>&1 || true
cat gpurun_out/r5b_km_ab_kernels.txt
