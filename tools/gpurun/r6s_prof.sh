#!/bin/bash
# round 6: kernel traces of the headline configs (1 GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6s/ts -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-validate > gpurun_out/r6s/ts.log 2>&1 || { tail -20 gpurun_out/r6s/ts.log; exit 1; }
cd benchmarks
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/r6s/gb -o run --output-format csv -- python3 groupby.py --steps 2 --warmup 1 --no-validate > ../gpurun_out/r6s/gb.log 2>&1 || { tail -20 ../gpurun_out/r6s/gb.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/r6s/join -o run --output-format csv -- python3 join.py --steps 2 --warmup 1 --no-validate > ../gpurun_out/r6s/join.log 2>&1 || { tail -20 ../gpurun_out/r6s/join.log; exit 1; }
cd ..
for k in ts gb join; do f=$(find gpurun_out/r6s/$k -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r6s/${k}_kernel_stats.csv; head -12 $f | cut -c1-160; done
