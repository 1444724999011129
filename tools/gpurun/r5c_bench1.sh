#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5c_bench1.log 2>&1 || { tail -20 gpurun_out/r5c_bench1.log; exit 1; }
grep -v "executor:" gpurun_out/r5c_bench1.log | tail -2 | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b1prof -o run -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r5c_bench1_prof.log 2>&1 || { tail -20 gpurun_out/r5c_bench1_prof.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py tests/test_gpu_terasort_stored.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c_b1_tests.log 2>&1 || { tail -30 gpurun_out/r5c_b1_tests.log; exit 1; }
tail -2 gpurun_out/r5c_b1_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5c_smoke.log 2>&1 || { tail -20 gpurun_out/r5c_smoke.log; exit 1; }
tail -1 gpurun_out/r5c_smoke.log
