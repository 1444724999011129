#!/bin/bash
# k-means assignment kernel: instruction mix and waits (PMC), in-tree library only
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export KM_AB_ONLY_IN_TREE=1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA \
  -d gpurun_out/pmc_km -o p1 --output-format csv -- python3 tools/micro/km_depth_ab.py > gpurun_out/pmc_km.log 2>&1 || { tail -5 gpurun_out/pmc_km.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
  -d gpurun_out/pmc_km -o p2 --output-format csv -- python3 tools/micro/km_depth_ab.py >> gpurun_out/pmc_km.log 2>&1 || { tail -5 gpurun_out/pmc_km.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 TA_TA_BUSY_sum \
  -d gpurun_out/pmc_km -o p3 --output-format csv -- python3 tools/micro/km_depth_ab.py >> gpurun_out/pmc_km.log 2>&1 || { tail -5 gpurun_out/pmc_km.log; echo "pass 3 counters unavailable"; }
grep -v amdgpu.ids gpurun_out/pmc_km.log | tail -6
