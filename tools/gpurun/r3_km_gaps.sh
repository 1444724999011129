#!/bin/bash
# Kernel timeline of the k-means benchmark (idle gaps between an iteration's kernels = host time).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R/benchmarks
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_kmg -o run -- python3 kmeans.py --iters 4 --warmup 1 \
  > $R/gpurun_out/prof_kmg.log 2>&1 || { tail -30 $R/gpurun_out/prof_kmg.log; exit 1; }
db=$(find $R/gpurun_out/prof_kmg -name '*.db' | head -1)
python3 $R/tools/trace_gaps.py "$db" --last 70 > $R/gpurun_out/gaps_km.txt
tail -75 $R/gpurun_out/gaps_km.txt
