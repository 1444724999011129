#!/bin/bash
# round 6: one box, every BASELINE config's benchmark, validated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6n
timeout -k 10 300 python -u bench.py > gpurun_out/r6n/bench.log 2>&1 || { tail -20 gpurun_out/r6n/bench.log; exit 1; }
tail -1 gpurun_out/r6n/bench.log | cut -c1-400
cd benchmarks
timeout -k 10 300 python3 -u groupby.py --steps 5 --warmup 1 > ../gpurun_out/r6n/groupby.log 2>&1 || { tail -20 ../gpurun_out/r6n/groupby.log; exit 1; }
tail -1 ../gpurun_out/r6n/groupby.log | cut -c1-400
timeout -k 10 400 python3 -u join.py --steps 3 --warmup 1 > ../gpurun_out/r6n/join.log 2>&1 || { tail -20 ../gpurun_out/r6n/join.log; exit 1; }
tail -1 ../gpurun_out/r6n/join.log | cut -c1-400
timeout -k 10 300 python3 -u kmeans.py > ../gpurun_out/r6n/kmeans.log 2>&1 || { tail -20 ../gpurun_out/r6n/kmeans.log; exit 1; }
tail -1 ../gpurun_out/r6n/kmeans.log | cut -c1-400
timeout -k 10 300 python3 -u wordcount.py --gpu --mb 1000 --partitions 1 > ../gpurun_out/r6n/wordcount.log 2>&1 || { tail -20 ../gpurun_out/r6n/wordcount.log; exit 1; }
tail -1 ../gpurun_out/r6n/wordcount.log | cut -c1-400
cd ..
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r6n/lb8.log 2>&1 || { tail -20 gpurun_out/r6n/lb8.log; exit 1; }
tail -1 gpurun_out/r6n/lb8.log | cut -c1-600
