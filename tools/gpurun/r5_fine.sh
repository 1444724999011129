#!/bin/bash
# round 5: fine-bucket exchange over materialised tables, streamed aggregation, loopback benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fine_rows.py tests/test_gpu_stream_agg.py -x -v --timeout 150 \
  --timeout-method thread > gpurun_out/r5_unit.log 2>&1 || { tail -60 gpurun_out/r5_unit.log; exit 1; }
tail -3 gpurun_out/r5_unit.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 580 --timeout-method thread \
  -k "fine_rows or two_ranks_share" > gpurun_out/r5_fine_multi.log 2>&1 || { tail -80 gpurun_out/r5_fine_multi.log; exit 1; }
tail -3 gpurun_out/r5_fine_multi.log
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r5_lb8_table.log 2>&1 \
  || { tail -30 gpurun_out/r5_lb8_table.log; exit 1; }
tail -2 gpurun_out/r5_lb8_table.log
