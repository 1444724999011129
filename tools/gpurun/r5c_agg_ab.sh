#!/bin/bash
# dense aggregation kernel grid (ops/densegroup.AGG_GRID) A/B on the 1-GPU GroupBy bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/benchmarks" || exit 1
mkdir -p ../gpurun_out
for g in 1024 2048 4096 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_agg_$g -o run --output-format csv -- \
    python3 -u groupby.py --steps 3 --warmup 1 --dg-agg-grid $g > ../gpurun_out/r5c_agg_$g.log 2>&1 || { tail -20 ../gpurun_out/r5c_agg_$g.log; exit 1; }
  echo "== $g $(grep -o '"ms_per_step": [0-9.]*\|"validated": [a-z]*' ../gpurun_out/r5c_agg_$g.log | tr '\n' ' ') $(grep dg_agg ../gpurun_out/prof_agg_$g/run_kernel_stats.csv | cut -d, -f3-5)"
done
