#!/bin/bash
# Rehearsal of the driver's 8-GPU bench path: 8 ranks share the one GPU over gloo, 5e7 records each
# (the fine-bucket exchange at W = 8: fb, rounds, tile merge of 8 source slices), validated across ranks.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export DRYAD_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29608 bench.py --gpus 8 --steps 2 --warmup 1 --records-per-gpu 50000000 --rehearsal \
  > gpurun_out/mr_bench_8.log 2>&1 || { tail -40 gpurun_out/mr_bench_8.log; exit 1; }
grep '"metric"' gpurun_out/mr_bench_8.log | cut -c1-900
