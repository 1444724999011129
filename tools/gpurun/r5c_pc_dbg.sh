#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 python -u tools/debug/pc_rows_dbg.py 2>&1 | grep -v amdgpu.ids
