#!/bin/bash
# Round-3 GPU check + a 2-rank gloo rehearsal of the driver's N>1 bench path on the one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_tests.log 2>&1 || { tail -60 gpurun_out/r3_tests.log; exit 1; }
tail -3 gpurun_out/r3_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench.log 2>&1 || { tail -30 gpurun_out/r3_bench.log; exit 1; }
grep '"metric"' gpurun_out/r3_bench.log | cut -c1-400
export DRYAD_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29602 bench.py --gpus 2 --steps 2 --warmup 1 --records-per-gpu 100000000 --rehearsal \
  > gpurun_out/mr_bench_2.log 2>&1 || { tail -40 gpurun_out/mr_bench_2.log; exit 1; }
grep '"metric"' gpurun_out/mr_bench_2.log | cut -c1-400
