#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/benchmarks" || exit 1
mkdir -p ../gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r5c_join -o run --output-format csv -- \
  python3 -u join.py --steps 2 --warmup 1 > ../gpurun_out/r5c_join.log 2>&1 || { tail -20 ../gpurun_out/r5c_join.log; exit 1; }
grep '"metric"' ../gpurun_out/r5c_join.log | cut -c1-300
