#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_oracle_suites.py -m gpu -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/oracle_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/oracle_gpu.log | tail -40
exit $rc
