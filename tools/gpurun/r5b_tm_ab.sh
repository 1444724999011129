#!/bin/bash
# tile merge A/B micro + PMC passes on the in-tree kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/micro/ts_merge_ab.py > gpurun_out/r5b_tm_ab.log 2>&1 || { tail -20 gpurun_out/r5b_tm_ab.log; exit 1; }
cat gpurun_out/r5b_tm_ab.log
for v in in-tree libtm_head.so; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
    -d gpurun_out/pmc_tm_$v -o p1 --output-format csv -- python3 tools/micro/ts_merge_ab.py $v > gpurun_out/pmc_tm_$v.log 2>&1 || { tail -5 gpurun_out/pmc_tm_$v.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -d gpurun_out/pmc_tm_$v -o p2 --output-format csv -- python3 tools/micro/ts_merge_ab.py $v >> gpurun_out/pmc_tm_$v.log 2>&1 || { tail -5 gpurun_out/pmc_tm_$v.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TA_BUSY_avr TA_TA_BUSY_sum \
    -d gpurun_out/pmc_tm_$v -o p3 --output-format csv -- python3 tools/micro/ts_merge_ab.py $v >> gpurun_out/pmc_tm_$v.log 2>&1 || { tail -5 gpurun_out/pmc_tm_$v.log; exit 1; }
done
ls gpurun_out/pmc_tm_in-tree
timeout -k 10 400 python -u tools/micro/writeback_probe2.py 15 /tmp/wbprobe2 > gpurun_out/r5b_writeback2.log 2>&1 || { tail -20 gpurun_out/r5b_writeback2.log; exit 1; }
cat gpurun_out/r5b_writeback2.log
