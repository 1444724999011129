#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd benchmarks
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d ../gpurun_out/prof_gbooc -o run --output-format csv -- \
  python3 -u groupby.py --records-per-gpu 1.5625e9 --hbm-budget-gb 20 --steps 1 --warmup 0 --no-validate > ../gpurun_out/r5_gbooc_prof.log 2>&1 || { tail -30 ../gpurun_out/r5_gbooc_prof.log; exit 1; }
grep '"metric"' ../gpurun_out/r5_gbooc_prof.log | cut -c1-300
head -25 ../gpurun_out/prof_gbooc/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
cat ../gpurun_out/prof_gbooc/run_memory_copy_stats.csv 2>/dev/null | cut -c1-200
