#!/bin/bash
# streamed GroupBy with the dense running state: tests, then 400 GB on one GPU under a 60 GB budget
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream_agg.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5c_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5c_dense_tests.log; exit 1; }
grep -c PASSED gpurun_out/r5c_dense_tests.log; tail -1 gpurun_out/r5c_dense_tests.log
cd benchmarks
timeout -k 10 600 python3 -u groupby.py --records-per-gpu 6.25e9 --hbm-budget-gb 60 --steps 1 --warmup 0 > ../gpurun_out/r5c_gb_ooc_dense.log 2>&1 || { tail -30 ../gpurun_out/r5c_gb_ooc_dense.log; exit 1; }
grep '"metric"' ../gpurun_out/r5c_gb_ooc_dense.log | cut -c1-1500
