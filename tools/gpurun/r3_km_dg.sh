#!/bin/bash
# k-means split planes + dense GroupBy: tests, then microbench / benches / profiles if they pass.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_hipgraph.py tests/test_gpu_densegroup.py -m gpu -q \
  --timeout 120 --timeout-method thread > gpurun_out/kmdg_tests.log 2>&1
rc=$?
tail -25 gpurun_out/kmdg_tests.log
# a crash / timeout ends the call; plain test failures still let the benches run
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/microbench_kmeans.py 125e6 64 > gpurun_out/km_micro.log 2>&1 || { tail -20 gpurun_out/km_micro.log; exit 1; }
cat gpurun_out/km_micro.log
timeout -k 10 300 python -u benchmarks/kmeans.py > gpurun_out/km_bench.log 2>&1 || { tail -30 gpurun_out/km_bench.log; exit 1; }
grep metric gpurun_out/km_bench.log | cut -c1-700
timeout -k 10 400 python -u benchmarks/groupby.py > gpurun_out/gb_bench.log 2>&1 || { tail -30 gpurun_out/gb_bench.log; exit 1; }
grep metric gpurun_out/gb_bench.log | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/km_prof -o km --output-format csv -- python3 benchmarks/kmeans.py --iters 3 \
  > gpurun_out/km_prof.log 2>&1 || { tail -20 gpurun_out/km_prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/gb_prof -o gb --output-format csv -- python3 benchmarks/groupby.py --steps 2 \
  > gpurun_out/gb_prof.log 2>&1 || { tail -20 gpurun_out/gb_prof.log; exit 1; }
find gpurun_out/km_prof gpurun_out/gb_prof -name "*kernel_stats.csv"
exit $rc
