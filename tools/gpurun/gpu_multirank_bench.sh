#!/bin/bash
# Rehearsal of the driver's multi-GPU bench on a one-GPU box: N ranks share the GPU over gloo
# (DRYAD_DIST_BACKEND=gloo), each sorting --records-per-gpu records through bench.py's N>1 path
# (sampled range partition, pipelined all-to-all-v, per-range sort + gather, cross-rank validation).
set -o pipefail
mkdir -p gpurun_out
export DRYAD_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 2 --warmup 1 --records-per-gpu 100000000 --rehearsal \
    > gpurun_out/mr_bench_$n.log 2>&1 || { tail -40 gpurun_out/mr_bench_$n.log; exit 1; }
  grep '"metric"' gpurun_out/mr_bench_$n.log
done
