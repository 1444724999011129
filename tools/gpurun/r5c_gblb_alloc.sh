#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/benchmarks" || exit 1
mkdir -p ../gpurun_out
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 4 --warmup 1 > ../gpurun_out/g_gblb8_exp.log 2>&1 || { tail -20 ../gpurun_out/g_gblb8_exp.log; exit 1; }
grep "step\|warmup" ../gpurun_out/g_gblb8_exp.log | cut -c1-120
