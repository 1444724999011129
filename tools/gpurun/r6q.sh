#!/bin/bash
# bench.py's N > 1 path end to end (JSON line, max over ranks, validation) as a shared-GPU gloo
# rehearsal at 2 and 4 ranks, small records per rank
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6q
for n in 2 4; do
  DRYAD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 2 --warmup 1 --records-per-gpu 30000000 --rehearsal > gpurun_out/r6q/bench_$n.log 2>&1 || { tail -30 gpurun_out/r6q/bench_$n.log; exit 1; }
  grep '"metric"' gpurun_out/r6q/bench_$n.log | cut -c1-700
done
