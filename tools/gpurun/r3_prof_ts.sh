#!/bin/bash
# rocprofv3 kernel statistics + timeline of the headline bench (3 timed steps).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ts2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 \
  > $R/gpurun_out/prof_ts2.log 2>&1 || { tail -30 $R/gpurun_out/prof_ts2.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_ts2.log | cut -c1-200
db=$(find $R/gpurun_out/prof_ts2 -name '*.db' | head -1)
python3 $R/tools/rocpd_summary.py "$db" --csv $R/gpurun_out/ts2_kernels.csv > /dev/null
cat $R/gpurun_out/ts2_kernels.csv | head -14
python3 $R/tools/trace_gaps.py "$db" --last 24 | tail -26
