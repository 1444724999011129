#!/bin/bash
# round 6, final tree: bench.py (TeraSort 125 GB), GroupBy and the hash join on one box, validated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zo
timeout -k 10 300 python -u bench.py > gpurun_out/r6zo/bench.log 2>&1 || { tail -20 gpurun_out/r6zo/bench.log; exit 1; }
tail -1 gpurun_out/r6zo/bench.log | cut -c1-300
cd benchmarks
timeout -k 10 300 python3 -u groupby.py --steps 5 --warmup 1 > ../gpurun_out/r6zo/groupby.log 2>&1 || { tail -20 ../gpurun_out/r6zo/groupby.log; exit 1; }
tail -1 ../gpurun_out/r6zo/groupby.log | cut -c1-300
timeout -k 10 400 python3 -u join.py --steps 3 --warmup 1 > ../gpurun_out/r6zo/join.log 2>&1 || { tail -20 ../gpurun_out/r6zo/join.log; exit 1; }
tail -1 ../gpurun_out/r6zo/join.log | cut -c1-300
timeout -k 10 300 python3 -u wordcount.py --gpu --mb 1000 --partitions 1 --steps 6 > ../gpurun_out/r6zo/wordcount.log 2>&1 || { tail -20 ../gpurun_out/r6zo/wordcount.log; exit 1; }
tail -1 ../gpurun_out/r6zo/wordcount.log | cut -c1-300
