#!/bin/bash
# PMC passes over the radix-aggregation fold kernel (GroupBy benchmark, radix path forced).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/benchmarks" || exit 1
mkdir -p ../gpurun_out/pmc_ra
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "ra_agg" \
    -d ../gpurun_out/pmc_ra/p$i -o run --output-format csv -- python3 groupby.py --steps 1 --warmup 0 \
    --no-validate --aggregation radix > ../gpurun_out/pmc_ra/p$i.log 2>&1 || { tail -5 ../gpurun_out/pmc_ra/p$i.log; exit 1; }
done
echo PMC_DONE
