#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/benchmarks" || exit 1
mkdir -p ../gpurun_out
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 3 --warmup 1 > ../gpurun_out/g_gblb8b.log 2>&1 || { tail -20 ../gpurun_out/g_gblb8b.log; exit 1; }
grep "step\|warmup" ../gpurun_out/g_gblb8b.log | cut -c1-120; grep '"metric"' ../gpurun_out/g_gblb8b.log | cut -c1-200
