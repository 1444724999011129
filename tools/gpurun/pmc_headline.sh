#!/bin/bash
# PMC passes over the headline TeraSort kernels (4e8 records) and the join kernels (12 GB tables):
# wave / instruction / LDS counters, then HBM bytes.  One counter group per rocprofv3 run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_h
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "gather_fixup|rs_scatter|rs_count|ts_gen" \
    -d gpurun_out/pmc_h/ts$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 \
    --records-per-gpu 400000000 --no-validate > gpurun_out/pmc_h/ts$i.log 2>&1 || { tail -5 gpurun_out/pmc_h/ts$i.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "gp_scatter|rp_scatter|rp_count|rj_join|gen_records64" \
    -d gpurun_out/pmc_h/jn$i -o run --output-format csv -- python3 benchmarks/join.py --table-gb 12 --steps 1 \
    --warmup 0 --no-validate > gpurun_out/pmc_h/jn$i.log 2>&1 || { tail -5 gpurun_out/pmc_h/jn$i.log; exit 1; }
done
echo PMC_DONE
