#!/bin/bash
# out-of-core GroupBy (streamed aggregation past the HBM budget) and the string-key grace join to
# a partfile at scale; SMALL=1: the same at a quarter / a fifth of the size
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "${SMALL:-0}" = 1 ]; then GB_ROWS=1.5625e9; GB_BUDGET=20; J_GB=10; J_BUDGET=4; TAG=small; else GB_ROWS=6.25e9; GB_BUDGET=60; J_GB=50; J_BUDGET=30; TAG=full; fi
cd benchmarks
timeout -k 10 ${GB_TIMEOUT:-500} python3 -u groupby.py --records-per-gpu $GB_ROWS --hbm-budget-gb $GB_BUDGET --steps 1 --warmup 0 \
  > ../gpurun_out/r5_gb_ooc_$TAG.log 2>&1 || { tail -30 ../gpurun_out/r5_gb_ooc_$TAG.log; exit 1; }
grep '"metric"' ../gpurun_out/r5_gb_ooc_$TAG.log | cut -c1-1500
free -g | head -2
rm -rf /tmp/jn; mkdir -p /tmp/jn
timeout -k 10 ${J_TIMEOUT:-500} python3 -u join.py --names --table-gb $J_GB --hbm-budget-gb $J_BUDGET --to-store partfile:///tmp/jn/out \
  --steps 1 --warmup 0 > ../gpurun_out/r5_join_names_$TAG.log 2>&1 || { tail -30 ../gpurun_out/r5_join_names_$TAG.log; exit 1; }
grep '"metric"' ../gpurun_out/r5_join_names_$TAG.log | cut -c1-2000
rm -rf /tmp/jn
