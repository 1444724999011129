#!/bin/bash
# round 6, mid-round check: GPU suite, smoke, 1-GPU bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6m_suite.log 2>&1 || { tail -40 gpurun_out/r6m_suite.log; exit 1; }
tail -1 gpurun_out/r6m_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6m_smoke.log 2>&1 || { tail -20 gpurun_out/r6m_smoke.log; exit 1; }
tail -1 gpurun_out/r6m_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6m_bench.log 2>&1 || { tail -20 gpurun_out/r6m_bench.log; exit 1; }
tail -1 gpurun_out/r6m_bench.log | cut -c1-300
