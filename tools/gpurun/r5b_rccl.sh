#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -k rccl \
  > gpurun_out/r5b_rccl.log 2>&1 || { tail -40 gpurun_out/r5b_rccl.log; cat gpurun_out/fail_rccl_one_rank.log 2>/dev/null | tail -40; exit 1; }
tail -3 gpurun_out/r5b_rccl.log
