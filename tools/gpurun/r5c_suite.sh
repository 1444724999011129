#!/bin/bash
# full GPU suite, then the headline bench and the 8-rank per-rank program
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c_suite.log 2>&1 || { tail -40 gpurun_out/r5c_suite.log; exit 1; }
tail -2 gpurun_out/r5c_suite.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5c_final_bench.log 2>&1 || { tail -20 gpurun_out/r5c_final_bench.log; exit 1; }
grep '"metric"' gpurun_out/r5c_final_bench.log | cut -c1-250
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r5c_final_lb8.log 2>&1 || { tail -20 gpurun_out/r5c_final_lb8.log; exit 1; }
tail -1 gpurun_out/r5c_final_lb8.log | cut -c1-250
