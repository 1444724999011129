#!/bin/bash
# round 6: full GPU suite + smoke (final kernel set: wide sorts incl. E256/E320 and the expand sort)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zm
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6zm/suite.log 2>&1 || { tail -40 gpurun_out/r6zm/suite.log; exit 1; }
tail -2 gpurun_out/r6zm/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6zm/smoke.log 2>&1 || { tail -20 gpurun_out/r6zm/smoke.log; exit 1; }
tail -2 gpurun_out/r6zm/smoke.log
