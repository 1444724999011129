#!/bin/bash
# round 6 (after the 16-wave workgroup kernels): one box, every BASELINE config, validated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zd
timeout -k 10 300 python -u bench.py > gpurun_out/r6zd/bench.log 2>&1 || { tail -20 gpurun_out/r6zd/bench.log; exit 1; }
tail -1 gpurun_out/r6zd/bench.log | cut -c1-400
cd benchmarks
timeout -k 10 300 python3 -u groupby.py --steps 5 --warmup 1 > ../gpurun_out/r6zd/groupby.log 2>&1 || { tail -20 ../gpurun_out/r6zd/groupby.log; exit 1; }
tail -1 ../gpurun_out/r6zd/groupby.log | cut -c1-400
timeout -k 10 400 python3 -u join.py --steps 3 --warmup 1 > ../gpurun_out/r6zd/join.log 2>&1 || { tail -20 ../gpurun_out/r6zd/join.log; exit 1; }
tail -1 ../gpurun_out/r6zd/join.log | cut -c1-400
timeout -k 10 300 python3 -u kmeans.py > ../gpurun_out/r6zd/kmeans.log 2>&1 || { tail -20 ../gpurun_out/r6zd/kmeans.log; exit 1; }
tail -1 ../gpurun_out/r6zd/kmeans.log | cut -c1-400
timeout -k 10 300 python3 -u wordcount.py --gpu --mb 1000 --partitions 1 > ../gpurun_out/r6zd/wordcount.log 2>&1 || { tail -20 ../gpurun_out/r6zd/wordcount.log; exit 1; }
tail -1 ../gpurun_out/r6zd/wordcount.log | cut -c1-400
cd ..
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r6zd/lb8.log 2>&1 || { tail -20 gpurun_out/r6zd/lb8.log; exit 1; }
tail -1 gpurun_out/r6zd/lb8.log | cut -c1-600
timeout -k 10 400 python -u bench.py --loopback-ranks 8 --loopback-table records64 --loopback-gb 80 --steps 2 --warmup 1 > gpurun_out/r6zd/r64_lb8.log 2>&1 || { tail -20 gpurun_out/r6zd/r64_lb8.log; exit 1; }
tail -1 gpurun_out/r6zd/r64_lb8.log | cut -c1-400
(cd benchmarks && timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 3 --warmup 1 --stream-shuffle --hbm-budget-gb 200 > ../gpurun_out/r6zd/gblb8_ss200.log 2>&1) || { tail -20 gpurun_out/r6zd/gblb8_ss200.log; exit 1; }
tail -1 gpurun_out/r6zd/gblb8_ss200.log | cut -c1-800
