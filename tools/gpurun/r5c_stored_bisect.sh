#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/_bisect" || exit 1
mkdir -p ../gpurun_out
timeout -k 10 200 python -u -X faulthandler -m pytest tests/test_gpu_terasort_stored.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > ../gpurun_out/r5c_stored_bisect.log 2>&1; echo "old tree rc=$?"
grep -E "PASS|FAIL|Fatal" ../gpurun_out/r5c_stored_bisect.log | head -5
