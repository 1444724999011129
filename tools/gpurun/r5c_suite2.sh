#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c_suite2.log 2>&1 || { tail -40 gpurun_out/r5c_suite2.log; exit 1; }
tail -2 gpurun_out/r5c_suite2.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5c_smoke2.log 2>&1 || { tail -20 gpurun_out/r5c_smoke2.log; exit 1; }
tail -1 gpurun_out/r5c_smoke2.log
