#!/bin/bash
# GPU check for gpurun: selected GPU tests, then the headline bench.  Each GPU step has its own
# time limit and the script stops at the first failure.
#   tools/gpu_check.sh "<pytest files>" [bench args]
set -o pipefail
mkdir -p gpurun_out
TESTS=${1:-tests}
shift
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
if [ "$1" != "nobench" ]; then
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -12 gpurun_out/bench.log
fi
