#!/bin/bash
# Kernel timeline of the headline bench (3 timed steps): idle gaps between kernels = host overhead.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_gaps -o run -- python3 $R/bench.py --steps 3 --warmup 1 \
  > $R/gpurun_out/prof_gaps.log 2>&1 || { tail -30 $R/gpurun_out/prof_gaps.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_gaps.log | cut -c1-300
db=$(find $R/gpurun_out/prof_gaps -name '*.db' | head -1)
python3 $R/tools/trace_gaps.py "$db" --last 80 > $R/gpurun_out/gaps_ts.txt
cat $R/gpurun_out/gaps_ts.txt | tail -90
