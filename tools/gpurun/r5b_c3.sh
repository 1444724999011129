#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --records-per-gpu 250000000 --input partfile:///tmp/ts_in --output partfile:///tmp/ts_out \
  --steps 4 --warmup 1 > gpurun_out/r5b_stored2.log 2>&1 || { tail -20 gpurun_out/r5b_stored2.log; exit 1; }
grep '"metric"' gpurun_out/r5b_stored2.log | grep -o '"stored": .*' | cut -c1-1200
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 600 --timeout-method thread -k "sweep" \
  > gpurun_out/r5b_sweep.log 2>&1 || { tail -40 gpurun_out/r5b_sweep.log; exit 1; }
tail -6 gpurun_out/r5b_sweep.log
