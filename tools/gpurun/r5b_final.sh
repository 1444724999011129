#!/bin/bash
# round-5 measurement set: headline bench, loopback per-rank programs, the BASELINE configs, smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/f_bench.log 2>&1 || { tail -20 gpurun_out/f_bench.log; exit 1; }
grep '"metric"' gpurun_out/f_bench.log | cut -c1-260
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/f_lb8.log 2>&1 || { tail -20 gpurun_out/f_lb8.log; exit 1; }
tail -1 gpurun_out/f_lb8.log | cut -c1-300
cd benchmarks
timeout -k 10 400 python3 -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/f_gb.log 2>&1 || { tail -20 ../gpurun_out/f_gb.log; exit 1; }
grep '"metric"' ../gpurun_out/f_gb.log | cut -c1-260
timeout -k 10 600 python3 -u join.py --steps 2 --warmup 1 > ../gpurun_out/f_join.log 2>&1 || { tail -20 ../gpurun_out/f_join.log; exit 1; }
grep '"metric"' ../gpurun_out/f_join.log | cut -c1-260
timeout -k 10 400 python3 -u kmeans.py > ../gpurun_out/f_km.log 2>&1 || { tail -20 ../gpurun_out/f_km.log; exit 1; }
grep '"metric"' ../gpurun_out/f_km.log | cut -c1-300
cd ..
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || { tail -20 gpurun_out/f_smoke.log; exit 1; }
tail -1 gpurun_out/f_smoke.log
