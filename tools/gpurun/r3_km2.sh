#!/bin/bash
# k-means (bf16 plane + kept sums) tests / microbench / bench / kernel trace, dense GroupBy tests,
# then PMC passes over the dense GroupBy kernels (one counter group per run).
set -o pipefail
mkdir -p gpurun_out/pmc_dg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans.py tests/test_gpu_hipgraph.py tests/test_gpu_densegroup.py -m gpu -q \
  --timeout 120 --timeout-method thread > gpurun_out/kmdg_tests.log 2>&1
rc=$?
tail -25 gpurun_out/kmdg_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/microbench_kmeans.py 125e6 64 > gpurun_out/km_micro.log 2>&1 || { tail -20 gpurun_out/km_micro.log; exit 1; }
cat gpurun_out/km_micro.log
timeout -k 10 300 python -u benchmarks/kmeans.py > gpurun_out/km_bench.log 2>&1 || { tail -30 gpurun_out/km_bench.log; exit 1; }
grep metric gpurun_out/km_bench.log | cut -c1-700
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/km_prof -o km --output-format csv -- python3 benchmarks/kmeans.py --iters 3 \
  > gpurun_out/km_prof.log 2>&1 || { tail -20 gpurun_out/km_prof.log; exit 1; }
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "dg_|kmeans_assign|kmeans_movers" \
    -d gpurun_out/pmc_dg/p$i -o run --output-format csv -- python3 benchmarks/groupby.py --steps 1 --warmup 0 --records-per-gpu 5e8 \
    > gpurun_out/pmc_dg/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_dg/p$i.log; echo "pass $i failed"; exit 1; }
done
echo PMC_DONE
exit $rc
