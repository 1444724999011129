#!/bin/bash
# round 6: page-locking cost with parallel prefault, GroupBy streamed shuffle (received partials
# held and reduced once) at a node-sized budget, 150 GB Distinct again
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/micro/pinned_alloc.py > gpurun_out/r6f_pinned.log 2>&1 || { tail -20 gpurun_out/r6f_pinned.log; exit 1; }
cat gpurun_out/r6f_pinned.log | grep GB
cd benchmarks
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 --stream-shuffle --hbm-budget-gb 200 > ../gpurun_out/r6f_gblb8_ss200.log 2>&1 || { tail -20 ../gpurun_out/r6f_gblb8_ss200.log; exit 1; }
tail -1 ../gpurun_out/r6f_gblb8_ss200.log | cut -c1-1500
timeout -k 10 600 python3 -u distinct.py --gb 150 --hbm-budget-gb 60 > ../gpurun_out/r6f_distinct150.log 2>&1 || { tail -20 ../gpurun_out/r6f_distinct150.log; exit 1; }
tail -1 ../gpurun_out/r6f_distinct150.log | cut -c1-2500
