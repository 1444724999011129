#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
DRYAD_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29701 tools/memprobe.py > gpurun_out/memprobe.log 2>&1 || { tail -30 gpurun_out/memprobe.log; exit 1; }
grep "\[mem\]" gpurun_out/memprobe.log
