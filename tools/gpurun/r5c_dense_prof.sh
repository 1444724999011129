#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/benchmarks" || exit 1
mkdir -p ../gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r5c_dense -o run --output-format csv -- \
  python3 -u groupby.py --records-per-gpu 1.5625e9 --hbm-budget-gb 60 --steps 1 --warmup 0 --no-validate > ../gpurun_out/r5c_dense_prof.log 2>&1 || { tail -30 ../gpurun_out/r5c_dense_prof.log; exit 1; }
grep '"metric"' ../gpurun_out/r5c_dense_prof.log | cut -c1-300
