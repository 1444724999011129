#!/bin/bash
# PMC passes over the k-means step kernel (microbench, 50M points, K = 64).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_km
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "kmeans_mfma" \
    -d gpurun_out/pmc_km/p$i -o run --output-format csv -- python3 tools/micro/microbench_kmeans.py 50e6 64 \
    > gpurun_out/pmc_km/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_km/p$i.log; echo "pass $i failed"; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_km/trace -o run --output-format csv -- python3 tools/micro/microbench_kmeans.py 50e6 64 > gpurun_out/pmc_km/trace.log 2>&1 || { echo trace failed; exit 1; }
echo PMC_DONE
