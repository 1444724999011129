#!/bin/bash
# per-rank program of the 8-GPU GroupBy under rocprofv3 (kernel CSV), with the HBM working set
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd benchmarks
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r5b_gblb -o run --output-format csv -- \
  python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/r5b_gblb.log 2>&1 || { tail -20 ../gpurun_out/r5b_gblb.log; exit 1; }
grep '"metric"' ../gpurun_out/r5b_gblb.log | cut -c1-1200
