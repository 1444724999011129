#!/bin/bash
# column bounds carried through partition / exchange / concat: GPU tests that shuffle device
# tables, then the 8-rank GroupBy loopback (stage B's min/max pass should be gone)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_stream_agg.py tests/test_gpu_densegroup.py tests/test_gpu_channel.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r5c_bounds_tests.log 2>&1 || { tail -40 gpurun_out/r5c_bounds_tests.log; exit 1; }
tail -1 gpurun_out/r5c_bounds_tests.log
cd benchmarks
timeout -k 10 300 python3 -u groupby.py --loopback-ranks 8 --steps 4 --warmup 1 > ../gpurun_out/r5c_bounds_gblb8.log 2>&1 || { tail -20 ../gpurun_out/r5c_bounds_gblb8.log; exit 1; }
grep "step" ../gpurun_out/r5c_bounds_gblb8.log | cut -c1-120
grep -o '"ms_per_step": [0-9.]*\|"validated": {"ok": [a-z]*' ../gpurun_out/r5c_bounds_gblb8.log | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r5c_bounds -o run --output-format csv -- \
  python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/r5c_bounds_prof.log 2>&1 || { tail -20 ../gpurun_out/r5c_bounds_prof.log; exit 1; }
