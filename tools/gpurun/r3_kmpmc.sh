#!/bin/bash
# PMC passes over the k-means assignment / movers kernels (125M x 128, K = 64), one group per run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_km3
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "kmeans_assign|kmeans_movers|kmeans_hi" \
    -d gpurun_out/pmc_km3/p$i -o run --output-format csv -- python3 tools/microbench_kmeans.py 125e6 64 \
    > gpurun_out/pmc_km3/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_km3/p$i.log; echo "pass $i failed"; exit 1; }
done
echo PMC_DONE
