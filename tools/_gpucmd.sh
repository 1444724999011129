#!/bin/bash
# scratch GPU command (gpurun): build, run the selected GPU tests
set -o pipefail
mkdir -p gpurun_out
python -m dryad_amd._build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests/test_gpu_fingerprint.py tests/test_gpu_executor.py -x -q -m gpu > gpurun_out/t.log 2>&1
rc=$?
tail -30 gpurun_out/t.log
exit $rc
