#!/bin/bash
# kernel profile of the loopback per-rank program (materialised table) + the GroupBy loopback
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5_lb -o run --output-format csv -- \
  python3 bench.py --loopback-ranks 8 --steps 2 --warmup 1 > gpurun_out/r5_lb8_prof.log 2>&1 || { tail -20 gpurun_out/r5_lb8_prof.log; exit 1; }
tail -1 gpurun_out/r5_lb8_prof.log | cut -c1-300
cd benchmarks
timeout -k 10 400 python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/r5_gb_lb8.log 2>&1 || { tail -20 ../gpurun_out/r5_gb_lb8.log; exit 1; }
tail -1 ../gpurun_out/r5_gb_lb8.log
timeout -k 10 400 python3 -u groupby.py --loopback-ranks 8 --raw-shuffle --steps 2 --warmup 1 > ../gpurun_out/r5_gb_lb8_raw.log 2>&1 || { tail -20 ../gpurun_out/r5_gb_lb8_raw.log; exit 1; }
tail -1 ../gpurun_out/r5_gb_lb8_raw.log
