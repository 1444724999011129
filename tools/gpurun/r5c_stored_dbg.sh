#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -X faulthandler -m pytest tests/test_gpu_terasort_stored.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r5c_stored_alone.log 2>&1; echo "alone rc=$?"
grep -E "PASS|FAIL|Fatal|Error" gpurun_out/r5c_stored_alone.log | head -10
