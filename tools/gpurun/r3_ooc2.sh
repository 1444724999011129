#!/bin/bash
# Out-of-core TeraSort after the sort-phase slot change: extsort tests, the 100 GB / 48 GB-budget
# point (3 timed steps), then the 400 GB 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_extsort.py -m gpu -q -x --timeout 200 --timeout-method thread \
  > gpurun_out/ooc_tests.log 2>&1 || { tail -40 gpurun_out/ooc_tests.log; exit 1; }
tail -2 gpurun_out/ooc_tests.log
timeout -k 10 400 python -u benchmarks/terasort_ooc.py --steps 3 > gpurun_out/ooc_100.log 2>&1 || { tail -20 gpurun_out/ooc_100.log; exit 1; }
grep "^\[ooc\] step" gpurun_out/ooc_100.log | cut -c1-400
tail -1 gpurun_out/ooc_100.log | cut -c1-600
timeout -k 10 600 python -u bench.py --total-bytes 4e11 --steps 2 --warmup 1 > gpurun_out/ooc_400.log 2>&1 || { tail -20 gpurun_out/ooc_400.log; exit 1; }
tail -1 gpurun_out/ooc_400.log | cut -c1-700
