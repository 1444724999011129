#!/bin/bash
# full GPU suite + headline bench + smoke + page-cache write-back probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5_full_tests.log 2>&1 || { tail -40 gpurun_out/r5_full_tests.log; exit 1; }
tail -2 gpurun_out/r5_full_tests.log
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r5_lb8.log 2>&1 || { tail -20 gpurun_out/r5_lb8.log; exit 1; }
tail -1 gpurun_out/r5_lb8.log | cut -c1-400
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5_bench.log 2>&1 || { tail -20 gpurun_out/r5_bench.log; exit 1; }
grep '"metric"' gpurun_out/r5_bench.log | cut -c1-300
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
timeout -k 10 400 python -u tools/micro/writeback_probe.py 25 /tmp/wbprobe > gpurun_out/r5_writeback.log 2>&1 || { tail -20 gpurun_out/r5_writeback.log; exit 1; }
cat gpurun_out/r5_writeback.log | cut -c1-200
