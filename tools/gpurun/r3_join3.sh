#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u benchmarks/join.py --hbm-budget-gb 30 --steps 3 > gpurun_out/r3_join_spill.log 2>&1 || { tail -30 gpurun_out/r3_join_spill.log; exit 1; }
grep '"metric"' gpurun_out/r3_join_spill.log | cut -c1-1500
