#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug/pc_rows_dbg.py 2>&1 | grep -v amdgpu.ids | head -8
timeout -k 10 300 python -u -m pytest tests/test_gpu_channel.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c_pc_tests.log 2>&1 || { tail -30 gpurun_out/r5c_pc_tests.log; exit 1; }
tail -2 gpurun_out/r5c_pc_tests.log
cd benchmarks
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r5c_gblb -o run --output-format csv -- \
  python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/r5c_gblb.log 2>&1 || { tail -20 ../gpurun_out/r5c_gblb.log; exit 1; }
grep '"metric"' ../gpurun_out/r5c_gblb.log | cut -c1-600
