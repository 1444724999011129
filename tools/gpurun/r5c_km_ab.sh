#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/micro/km_depth_ab.py > gpurun_out/r5c_km_ab.log 2>&1 || { tail -20 gpurun_out/r5c_km_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5c_km_ab.log | tail -8
