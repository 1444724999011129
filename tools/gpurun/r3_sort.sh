#!/bin/bash
# E64 scatter variants A/B, sort tests, TeraSort bench + kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u tools/microbench_sort64.py 1000000000 > gpurun_out/sort64_ab.log 2>&1 || { tail -20 gpurun_out/sort64_ab.log; exit 1; }
cat gpurun_out/sort64_ab.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "sort or terasort or extsort or recordsort" --timeout 200 --timeout-method thread \
  > gpurun_out/sort_tests.log 2>&1 || { tail -30 gpurun_out/sort_tests.log; exit 1; }
tail -2 gpurun_out/sort_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ts_bench.log 2>&1 || { tail -20 gpurun_out/ts_bench.log; exit 1; }
grep metric gpurun_out/ts_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ts_prof -o ts --output-format csv -- python3 bench.py --steps 3 --warmup 1 \
  > gpurun_out/ts_prof.log 2>&1 || { tail -20 gpurun_out/ts_prof.log; exit 1; }
echo DONE
