#!/bin/bash
# PMC pass over the partition / radix scatter kernels of a reduced join (one counter group per
# rocprofv3 run, kernel filter by regex).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_sc
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "${REGEX:-rp_scatter|gp_scatter|rs_scatter}" \
    -d gpurun_out/pmc_sc/p$i -o run --output-format csv -- python3 benchmarks/join.py --table-gb 12 --steps 1 \
    --warmup 0 --no-validate > gpurun_out/pmc_sc/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_sc/p$i.log; exit 1; }
done
echo PMC_DONE
