#!/bin/bash
# round 6: full GPU suite + smoke (final tree: wide sorts off)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zn
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6zn/suite.log 2>&1 || { tail -40 gpurun_out/r6zn/suite.log; exit 1; }
tail -2 gpurun_out/r6zn/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6zn/smoke.log 2>&1 || { tail -20 gpurun_out/r6zn/smoke.log; exit 1; }
tail -2 gpurun_out/r6zn/smoke.log
