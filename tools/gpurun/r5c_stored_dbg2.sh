#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug/stored_steps.py 3e6 > gpurun_out/r5c_stored_dbg2.log 2>&1; echo "rc=$?"
grep -v "^  File\|^Thread\|^$" gpurun_out/r5c_stored_dbg2.log | head -30 | cut -c1-200
