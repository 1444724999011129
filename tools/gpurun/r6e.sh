#!/bin/bash
# round 6: one-key bucket copy, records64 descending at 80 GB, out-of-core OrderByDescending past
# HBM, 150 GB all-distinct Distinct to host:// under a 60 GB budget
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tsmerge.py tests/test_gpu_fine_rows.py tests/test_gpu_stream_shuffle.py tests/test_gpu_stream_agg.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1 || { tail -60 gpurun_out/r6e_tests.log; exit 1; }
tail -1 gpurun_out/r6e_tests.log
(cd benchmarks && timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 --stream-shuffle > ../gpurun_out/r6e_gblb8_ss.log 2>&1) || { tail -20 gpurun_out/r6e_gblb8_ss.log; exit 1; }
tail -1 gpurun_out/r6e_gblb8_ss.log | cut -c1-1500
timeout -k 10 400 python -u bench.py --loopback-ranks 8 --loopback-table records64 --loopback-gb 80 --sort-key Key --descending --steps 2 --warmup 1 > gpurun_out/r6e_r64_lb8_desc.log 2>&1 || { tail -20 gpurun_out/r6e_r64_lb8_desc.log; exit 1; }
tail -1 gpurun_out/r6e_r64_lb8_desc.log | cut -c1-1500
timeout -k 10 600 python -u bench.py --total-bytes 150e9 --descending --steps 1 --warmup 0 > gpurun_out/r6e_ooc_desc150.log 2>&1 || { tail -20 gpurun_out/r6e_ooc_desc150.log; exit 1; }
tail -1 gpurun_out/r6e_ooc_desc150.log | cut -c1-2500
free -g > gpurun_out/r6e_free.txt
cd benchmarks
timeout -k 10 600 python3 -u distinct.py --gb 150 --hbm-budget-gb 60 > ../gpurun_out/r6e_distinct150.log 2>&1 || { tail -20 ../gpurun_out/r6e_distinct150.log; exit 1; }
tail -1 ../gpurun_out/r6e_distinct150.log | cut -c1-2500
timeout -k 10 600 python3 -u join.py --to-store partfile:///tmp/dryad_jout --steps 2 --warmup 1 > ../gpurun_out/r6e_join_store.log 2>&1 || { tail -20 ../gpurun_out/r6e_join_store.log; exit 1; }
tail -1 ../gpurun_out/r6e_join_store.log | cut -c1-2500
rm -rf /tmp/dryad_jout*
timeout -k 10 600 python3 -u join.py --names --name-len 200 --table-gb 20 --to-store partfile:///tmp/dryad_jnames --steps 2 --warmup 1 > ../gpurun_out/r6e_join_names200.log 2>&1 || { tail -20 ../gpurun_out/r6e_join_names200.log; exit 1; }
tail -1 ../gpurun_out/r6e_join_names200.log | cut -c1-2500
