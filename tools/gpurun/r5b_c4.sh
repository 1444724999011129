#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --records-per-gpu 250000000 --input partfile:///tmp/ts_in --output partfile:///tmp/ts_out \
  --steps 4 --warmup 1 > gpurun_out/r5b_stored3.log 2>&1 || { tail -20 gpurun_out/r5b_stored3.log; exit 1; }
grep '"metric"' gpurun_out/r5b_stored3.log | grep -o '"value": [0-9.]*\|"job_phases_s": {[^}]*}\|"submit_and_wait_s": {[^}]*}'
rm -rf /tmp/ts_in* /tmp/ts_out*
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5b_full_tests.log 2>&1 || { tail -40 gpurun_out/r5b_full_tests.log; exit 1; }
tail -2 gpurun_out/r5b_full_tests.log
