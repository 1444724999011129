#!/bin/bash
# PMC passes over the E64 radix count / scatter kernels (one counter group per rocprofv3 run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc64
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc64/avail.txt 2>&1 || true
grep -o "TCC_EA0_W[A-Z0-9_]*\|TCC_W[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*\|TCC_PROBE[A-Z0-9_]*" gpurun_out/pmc64/avail.txt | sort -u | head -40
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex "rs_scatter|rs_count" \
    -d gpurun_out/pmc64/p$i -o run --output-format csv -- python3 tools/pmc_sort64_once.py 400000000 \
    > gpurun_out/pmc64/p$i.log 2>&1 || { tail -5 gpurun_out/pmc64/p$i.log; exit 1; }
done
echo PMC_DONE
