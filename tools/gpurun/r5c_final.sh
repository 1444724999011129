#!/bin/bash
# round-5 final measurement set (session 3): headline bench, per-rank programs, BASELINE configs, stored, RCCL rehearsal
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/g_bench.log 2>&1 || { tail -20 gpurun_out/g_bench.log; exit 1; }
grep '"metric"' gpurun_out/g_bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/g_lb8.log 2>&1 || { tail -20 gpurun_out/g_lb8.log; exit 1; }
tail -1 gpurun_out/g_lb8.log | cut -c1-200
timeout -k 10 500 python -u bench.py --rccl-one-rank --steps 3 --warmup 1 > gpurun_out/g_rccl1.log 2>&1 || { tail -20 gpurun_out/g_rccl1.log; exit 1; }
grep '"metric"' gpurun_out/g_rccl1.log | cut -c1-200
cd benchmarks
timeout -k 10 400 python3 -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/g_gb.log 2>&1 || { tail -20 ../gpurun_out/g_gb.log; exit 1; }
grep '"metric"' ../gpurun_out/g_gb.log | cut -c1-200
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/g_gblb8.log 2>&1 || { tail -20 ../gpurun_out/g_gblb8.log; exit 1; }
grep '"metric"' ../gpurun_out/g_gblb8.log | cut -c1-200
timeout -k 10 600 python3 -u join.py --steps 2 --warmup 1 > ../gpurun_out/g_join.log 2>&1 || { tail -20 ../gpurun_out/g_join.log; exit 1; }
grep '"metric"' ../gpurun_out/g_join.log | cut -c1-200
timeout -k 10 400 python3 -u kmeans.py > ../gpurun_out/g_km.log 2>&1 || { tail -20 ../gpurun_out/g_km.log; exit 1; }
grep '"metric"' ../gpurun_out/g_km.log | cut -c1-200
