#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tsmerge.py tests/test_gpu_fine_rows.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c_fs_tests.log 2>&1 || { tail -30 gpurun_out/r5c_fs_tests.log; exit 1; }
tail -1 gpurun_out/r5c_fs_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5c_fs -o run --output-format csv -- python3 -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r5c_fs_lb8.log 2>&1 || { tail -20 gpurun_out/r5c_fs_lb8.log; exit 1; }
grep "step 2" gpurun_out/r5c_fs_lb8.log | cut -c1-250; tail -1 gpurun_out/r5c_fs_lb8.log | grep -o '"validated": [a-z]*'
