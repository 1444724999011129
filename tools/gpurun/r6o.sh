#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6o
cd benchmarks
timeout -k 10 300 python3 -u wordcount.py --gpu --mb 1000 --partitions 1 --steps 6 > ../gpurun_out/r6o/wc.log 2>&1 || { tail -20 ../gpurun_out/r6o/wc.log; exit 1; }
tail -1 ../gpurun_out/r6o/wc.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/r6o/prof -o run --output-format csv -- python3 wordcount.py --gpu --mb 1000 --partitions 1 --steps 3 > ../gpurun_out/r6o/wc_prof.log 2>&1 || { tail -20 ../gpurun_out/r6o/wc_prof.log; exit 1; }
head -12 $(find ../gpurun_out/r6o/prof -name "*kernel_stats.csv" | head -1) | cut -c1-200
