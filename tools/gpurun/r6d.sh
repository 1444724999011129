#!/bin/bash
# round 6: vectorised per-round merge args, 2 receive slots (one in the table tail), pack-group A/B,
# kernel trace of the 8-rank loopback, one-rank RCCL peak, GroupBy loopback (bulk vs streamed
# shuffle, modelled link), small out-of-core Distinct to host://
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rowpack.py tests/test_gpu_tsmerge.py tests/test_gpu_fine_rows.py tests/test_gpu_multirank.py tests/test_gpu_extsort.py -x -q --timeout 580 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1 || { tail -60 gpurun_out/r6d_tests.log; exit 1; }
tail -1 gpurun_out/r6d_tests.log
timeout -k 10 400 python -u bench.py --loopback-ranks 8 --loopback-table records64 --loopback-gb 80 --steps 2 --warmup 1 > gpurun_out/r6d_r64_lb8.log 2>&1 || { tail -20 gpurun_out/r6d_r64_lb8.log; exit 1; }
tail -1 gpurun_out/r6d_r64_lb8.log | cut -c1-1800
timeout -k 10 400 python -u bench.py --loopback-ranks 8 --loopback-table records64 --loopback-gb 80 --sort-key Key --descending --steps 2 --warmup 1 > gpurun_out/r6d_r64_lb8_desc.log 2>&1 || { tail -20 gpurun_out/r6d_r64_lb8_desc.log; exit 1; }
tail -1 gpurun_out/r6d_r64_lb8_desc.log | cut -c1-1800
for g in 1 2; do
timeout -k 10 300 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 --pack-group $g > gpurun_out/r6d_lb8_g$g.log 2>&1 || { tail -20 gpurun_out/r6d_lb8_g$g.log; exit 1; }
tail -1 gpurun_out/r6d_lb8_g$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('group $g', d['value'], c['phases_ms'], c['validated'], c['modelled_exchange'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6d_lb8 -o run --output-format csv -- python3 bench.py --loopback-ranks 8 --steps 1 --warmup 1 > gpurun_out/r6d_lb8_prof.log 2>&1 || { tail -20 gpurun_out/r6d_lb8_prof.log; exit 1; }
find gpurun_out/prof_r6d_lb8 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -25 {}' > gpurun_out/r6d_lb8_kernel_stats.txt
cat gpurun_out/r6d_lb8_kernel_stats.txt | cut -c1-200
timeout -k 10 400 python -u bench.py --rccl-one-rank --steps 2 --warmup 1 > gpurun_out/r6d_rccl1.log 2>&1 || { tail -20 gpurun_out/r6d_rccl1.log; exit 1; }
tail -1 gpurun_out/r6d_rccl1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['validated'], c['hbm_peak_allocated_GB'], c['hbm_free_after_step_GB'], c['exchange'].get('overlap'), c['exchange'].get('first_round_queued_ms'))"
cd benchmarks
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/r6d_gblb8_bulk.log 2>&1 || { tail -20 ../gpurun_out/r6d_gblb8_bulk.log; exit 1; }
tail -1 ../gpurun_out/r6d_gblb8_bulk.log | cut -c1-1500
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 --stream-shuffle > ../gpurun_out/r6d_gblb8_ss.log 2>&1 || { tail -20 ../gpurun_out/r6d_gblb8_ss.log; exit 1; }
tail -1 ../gpurun_out/r6d_gblb8_ss.log | cut -c1-1500
timeout -k 10 300 python3 -u distinct.py --gb 10 --hbm-budget-gb 4 > ../gpurun_out/r6d_distinct10.log 2>&1 || { tail -20 ../gpurun_out/r6d_distinct10.log; exit 1; }
tail -1 ../gpurun_out/r6d_distinct10.log | cut -c1-1500
