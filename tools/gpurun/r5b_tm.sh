#!/bin/bash
# staged tile merge: numerics, then the loopback per-rank program under rocprofv3, then the write-back probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tsmerge.py tests/test_gpu_fine_rows.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5b_tm_tests.log 2>&1 || { tail -40 gpurun_out/r5b_tm_tests.log; exit 1; }
tail -2 gpurun_out/r5b_tm_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5b_lb -o run --output-format csv -- \
  python3 bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r5b_lb8.log 2>&1 || { tail -20 gpurun_out/r5b_lb8.log; exit 1; }
grep '\[bench\]' gpurun_out/r5b_lb8.log | cut -c1-300
timeout -k 10 400 python -u tools/micro/writeback_probe.py 15 /tmp/wbprobe > gpurun_out/r5b_writeback.log 2>&1 || { tail -20 gpurun_out/r5b_writeback.log; exit 1; }
cut -c1-200 gpurun_out/r5b_writeback.log
