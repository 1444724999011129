#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pitch128.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5c_bk_tests.log 2>&1 || { tail -40 gpurun_out/r5c_bk_tests.log; exit 1; }
tail -2 gpurun_out/r5c_bk_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bkab2 -o run -- python3 -u tools/micro/bucket_ab.py > gpurun_out/r5c_bucket_ab2.log 2>&1 || { tail -20 gpurun_out/r5c_bucket_ab2.log; exit 1; }
grep bucket= gpurun_out/r5c_bucket_ab2.log | cut -c1-120
f=$(find gpurun_out/bkab2 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -4 | cut -c1-60,200-
