#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 280 --timeout-method thread -k "two_ranks" > gpurun_out/r3_mr1.log 2>&1; tail -5 gpurun_out/r3_mr1.log
