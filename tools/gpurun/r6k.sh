#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stored_bounds.py -q --timeout 880 --timeout-method thread > gpurun_out/r6k_tests.log 2>&1; tail -30 gpurun_out/r6k_tests.log | cut -c1-3000
