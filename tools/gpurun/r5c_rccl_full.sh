#!/bin/bash
# one-rank RCCL rehearsal: the small test, then bench.py's multi-rank program at the full 125 GB per GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -k rccl \
  > gpurun_out/r5c_rccl.log 2>&1 || { tail -40 gpurun_out/r5c_rccl.log; tail -60 gpurun_out/fail_rccl_one_rank.log 2>/dev/null; exit 1; }
tail -3 gpurun_out/r5c_rccl.log
timeout -k 10 500 python -u bench.py --rccl-one-rank --steps 3 --warmup 1 > gpurun_out/r5c_rccl_bench.log 2>&1 || { tail -30 gpurun_out/r5c_rccl_bench.log; exit 1; }
grep -v "^\[bench\] executor" gpurun_out/r5c_rccl_bench.log | tail -8 | cut -c1-1500
