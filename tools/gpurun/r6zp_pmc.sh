#!/bin/bash
# round 6 PMC of the reshaped kernels: look-back scatter (1024 x 16) on the onesweep micro, dense
# GroupBy partition passes (8192-row tiles) and aggregation (1024 threads) on a 1-step GroupBy bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "os_scatter" -d gpurun_out/r6zp/os$i -o run --output-format csv -- \
    python3 tools/micro/onesweep_shape_ab.py 4e8 > gpurun_out/r6zp/os$i.log 2>&1 || { tail -5 gpurun_out/r6zp/os$i.log; exit 1; }
  (cd benchmarks && timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-include-regex "dg_scatter|dg_agg" -d ../gpurun_out/r6zp/dg$i -o run --output-format csv -- \
    python3 groupby.py --steps 1 --warmup 0 --no-validate > ../gpurun_out/r6zp/dg$i.log 2>&1) || { tail -5 gpurun_out/r6zp/dg$i.log; exit 1; }
  echo "pass $i done"
done
