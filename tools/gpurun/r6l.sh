#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest "tests/test_gpu_multirank.py::test_fine_rows_ranks_share_one_gpu[8]" -v --timeout 980 --timeout-method thread > gpurun_out/r6l_tests.log 2>&1; tail -5 gpurun_out/r6l_tests.log | cut -c1-3000
