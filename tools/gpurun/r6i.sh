#!/bin/bash
# round 6: look-back scatter ranking A/B (LDS atomicOr masks vs ballot match), kernel trace + PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6i
timeout -k 10 200 python -u tools/micro/onesweep_match_ab.py > gpurun_out/r6i/ab.log 2>&1 || { tail -20 gpurun_out/r6i/ab.log; exit 1; }
cat gpurun_out/r6i/ab.log | grep -v amdgpu.ids
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6i/trace -o run --output-format csv -- python3 tools/micro/onesweep_match_ab.py > gpurun_out/r6i/trace.log 2>&1 || { tail -20 gpurun_out/r6i/trace.log; exit 1; }
f=$(find gpurun_out/r6i/trace -name "*kernel_stats.csv" | head -1)
grep -E "os_scatter|os_hist" $f | cut -c1-260
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex "os_scatter" -d gpurun_out/r6i/pmc$i -o run --output-format csv -- python3 tools/micro/onesweep_match_ab.py 4e8 > gpurun_out/r6i/pmc$i.log 2>&1 || { tail -5 gpurun_out/r6i/pmc$i.log; exit 1; }
done
echo pmc done
