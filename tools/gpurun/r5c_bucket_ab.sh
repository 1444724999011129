#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/micro/bucket_ab.py > gpurun_out/r5c_bucket_ab.log 2>&1 || { tail -20 gpurun_out/r5c_bucket_ab.log; exit 1; }
cat gpurun_out/r5c_bucket_ab.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bkab -o run -- python3 -u tools/micro/bucket_ab.py > gpurun_out/r5c_bucket_ab_prof.log 2>&1 || { tail -20 gpurun_out/r5c_bucket_ab_prof.log; exit 1; }
f=$(find gpurun_out/bkab -name "*kernel_stats.csv" | head -1); cut -d, -f1-6 "$f" | head -14
