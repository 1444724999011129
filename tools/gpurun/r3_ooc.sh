#!/bin/bash
# Out-of-core TeraSort: extsort tests, the 100 GB / 48 GB-budget point (hybrid), then the largest
# 1-GPU input this box's host-memory cap allows through bench.py --total-bytes.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_extsort.py -m gpu -q -x --timeout 200 --timeout-method thread \
  > gpurun_out/ooc_tests.log 2>&1 || { tail -40 gpurun_out/ooc_tests.log; exit 1; }
tail -2 gpurun_out/ooc_tests.log
timeout -k 10 400 python -u benchmarks/terasort_ooc.py > gpurun_out/ooc_100.log 2>&1 || { tail -20 gpurun_out/ooc_100.log; exit 1; }
grep -v "^\[ooc\] step" gpurun_out/ooc_100.log | tail -3 | cut -c1-900
timeout -k 10 600 python -u bench.py --total-bytes 4e11 --steps 2 --warmup 1 > gpurun_out/ooc_400.log 2>&1 || { tail -20 gpurun_out/ooc_400.log; exit 1; }
tail -3 gpurun_out/ooc_400.log | cut -c1-1500
