#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --records-per-gpu 250000000 --input partfile:///tmp/ts_in --output partfile:///tmp/ts_out \
  --steps 6 --warmup 1 > gpurun_out/r5b_stored4.log 2>&1 || { tail -20 gpurun_out/r5b_stored4.log; exit 1; }
grep '"metric"' gpurun_out/r5b_stored4.log | grep -o '"value": [0-9.]*\|"steps": \[[^]]*\]'
rm -rf /tmp/ts_in* /tmp/ts_out*
bash tools/gpurun/gpu_multirank_bench.sh
