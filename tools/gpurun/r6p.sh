#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream_shuffle.py tests/test_gpu_stream_agg.py tests/test_gpu_multirank.py -q --timeout 880 --timeout-method thread > gpurun_out/r6p_tests.log 2>&1 || { tail -40 gpurun_out/r6p_tests.log; exit 1; }
tail -1 gpurun_out/r6p_tests.log
cd benchmarks
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 3 --warmup 1 --stream-shuffle --hbm-budget-gb 200 > ../gpurun_out/r6p_gblb8_ss200.log 2>&1 || { tail -20 ../gpurun_out/r6p_gblb8_ss200.log; exit 1; }
tail -1 ../gpurun_out/r6p_gblb8_ss200.log | cut -c1-1500
