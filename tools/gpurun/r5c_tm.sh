#!/bin/bash
# tile merge with the next bucket's rows prefetched: micro A/B vs the previous kernel, tests, loopback 8 ranks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/micro/ts_merge_ab.py in-tree libtm_head.so in-tree > gpurun_out/r5c_tm_ab.log 2>&1 || { tail -20 gpurun_out/r5c_tm_ab.log; exit 1; }
cat gpurun_out/r5c_tm_ab.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_tsmerge.py tests/test_gpu_fine_rows.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c_tm_tests.log 2>&1 || { tail -30 gpurun_out/r5c_tm_tests.log; exit 1; }
tail -2 gpurun_out/r5c_tm_tests.log
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r5c_lb8.log 2>&1 || { tail -20 gpurun_out/r5c_lb8.log; exit 1; }
grep "step" gpurun_out/r5c_lb8.log | cut -c1-250; tail -1 gpurun_out/r5c_lb8.log | cut -c1-600
