#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream_shuffle.py tests/test_gpu_pinned_pool.py tests/test_gpu_stream_agg.py -x -v --timeout 880 --timeout-method thread > gpurun_out/r6h_tests.log 2>&1 || { tail -60 gpurun_out/r6h_tests.log; exit 1; }
tail -3 gpurun_out/r6h_tests.log
