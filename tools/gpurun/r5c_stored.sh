#!/bin/bash
# stored-data TeraSort (partfile in -> sort -> partfile out, 25 GB) with recycled output parts
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --records-per-gpu 250000000 --input partfile:///tmp/ts_in --output partfile:///tmp/ts_out \
  --steps 5 --warmup 1 > gpurun_out/r5c_stored.log 2>&1 || { tail -20 gpurun_out/r5c_stored.log; exit 1; }
grep -v '^W20\|amdgpu.ids' gpurun_out/r5c_stored.log | cut -c1-1500
