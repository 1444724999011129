#!/bin/bash
# final tree: bench.py's N > 1 path as a shared-GPU gloo rehearsal at 2 and 4 ranks, and the one-rank
# RCCL rehearsal of the multi-rank program at the full 125 GB per rank
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zq
for n in 2 4; do
  DRYAD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 2 --warmup 1 --records-per-gpu 30000000 --rehearsal > gpurun_out/r6zq/bench_$n.log 2>&1 || { tail -30 gpurun_out/r6zq/bench_$n.log; exit 1; }
  grep '"metric"' gpurun_out/r6zq/bench_$n.log | cut -c1-400
done
timeout -k 10 400 python -u bench.py --rccl-one-rank --steps 2 --warmup 1 > gpurun_out/r6zq/rccl1.log 2>&1 || { tail -20 gpurun_out/r6zq/rccl1.log; exit 1; }
grep '"metric"' gpurun_out/r6zq/rccl1.log | cut -c1-400
grep -o '"validated": [a-z]*\|"hbm_free_after_step_GB": [0-9.]*' gpurun_out/r6zq/rccl1.log
