#!/bin/bash
# one-rank bucket sort (3 look-back passes + bucket gather): tests, then the headline bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pitch128.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5c_bk_tests.log 2>&1 || { tail -40 gpurun_out/r5c_bk_tests.log; exit 1; }
tail -3 gpurun_out/r5c_bk_tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r5c_bk_bench.log 2>&1 || { tail -20 gpurun_out/r5c_bk_bench.log; exit 1; }
grep -v "executor:" gpurun_out/r5c_bk_bench.log | tail -4 | cut -c1-400
grep -o '"path": "[^"]*"' gpurun_out/r5c_bk_bench.log | head -3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/bkprof -o run -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r5c_bk_prof.log 2>&1 || { tail -20 gpurun_out/r5c_bk_prof.log; exit 1; }
find gpurun_out/bkprof -name "*kernel_stats.csv" | head -2
