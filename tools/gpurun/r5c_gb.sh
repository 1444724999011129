#!/bin/bash
# dense GroupBy scatter at two workgroups per CU: numerics, then the 1-GPU GroupBy bench under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_densegroup.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5c_gb_tests.log 2>&1 || { tail -40 gpurun_out/r5c_gb_tests.log; exit 1; }
tail -2 gpurun_out/r5c_gb_tests.log
cd benchmarks
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r5c_gb -o run --output-format csv -- \
  python3 groupby.py --steps 3 --warmup 1 > ../gpurun_out/r5c_gb.log 2>&1 || { tail -20 ../gpurun_out/r5c_gb.log; exit 1; }
grep '"metric"' ../gpurun_out/r5c_gb.log | cut -c1-400
f=$(ls ../gpurun_out/prof_r5c_gb/*kernel_stats.csv | head -1); cut -d, -f1-4 "$f" | head -6 | cut -c1-60,150-
