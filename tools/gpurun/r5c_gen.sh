#!/bin/bash
# column generator (two rows per lane, 16-byte stores): numerics, then the 1-GPU GroupBy bench and
# the 8-rank loopback under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_grace.py tests/test_gpu_densegroup.py tests/test_gpu_stream_agg.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c_gen_tests.log 2>&1 || { tail -40 gpurun_out/r5c_gen_tests.log; exit 1; }
tail -1 gpurun_out/r5c_gen_tests.log
cd benchmarks
timeout -k 10 300 python3 -u groupby.py --steps 5 --warmup 1 > ../gpurun_out/r5c_gen_gb.log 2>&1 || { tail -20 ../gpurun_out/r5c_gen_gb.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"validated": [a-z]*' ../gpurun_out/r5c_gen_gb.log | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r5c_gen -o run --output-format csv -- \
  python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/r5c_gen_prof.log 2>&1 || { tail -20 ../gpurun_out/r5c_gen_prof.log; exit 1; }
grep "step" ../gpurun_out/r5c_gen_prof.log | cut -c1-110
