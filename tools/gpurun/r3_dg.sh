#!/bin/bash
# dense GroupBy: tests, the BASELINE GroupBy bench, a kernel-trace profile and a WRITE_SIZE pass.
set -o pipefail
mkdir -p gpurun_out/pmc_dg2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_densegroup.py tests/test_gpu_executor.py -m gpu -q -x \
  --timeout 120 --timeout-method thread > gpurun_out/dg_tests.log 2>&1 || { tail -40 gpurun_out/dg_tests.log; exit 1; }
tail -2 gpurun_out/dg_tests.log
timeout -k 10 400 python -u benchmarks/groupby.py > gpurun_out/gb_bench.log 2>&1 || { tail -30 gpurun_out/gb_bench.log; exit 1; }
grep metric gpurun_out/gb_bench.log | cut -c1-900
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/gb_prof -o gb --output-format csv -- python3 benchmarks/groupby.py --steps 2 \
  > gpurun_out/gb_prof.log 2>&1 || { tail -20 gpurun_out/gb_prof.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dg_|gen_records" \
  -d gpurun_out/pmc_dg2/w -o run --output-format csv -- python3 benchmarks/groupby.py --steps 1 --warmup 0 --records-per-gpu 5e8 \
  > gpurun_out/pmc_dg2/w.log 2>&1 || { tail -5 gpurun_out/pmc_dg2/w.log; echo "pmc failed"; exit 1; }
echo DONE
