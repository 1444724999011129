#!/bin/bash
# round 6: stored column bounds, JSON control gathers, GroupBy from host:// and partfile:// sources
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_stored_bounds.py tests/test_gpu_stream_shuffle.py tests/test_gpu_executor.py -q --timeout 880 --timeout-method thread > gpurun_out/r6j_tests.log 2>&1; rc=$?; tail -30 gpurun_out/r6j_tests.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
tail -1 gpurun_out/r6j_tests.log
cd benchmarks
timeout -k 10 300 python3 -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/r6j_gb_gen.log 2>&1 || { tail -20 ../gpurun_out/r6j_gb_gen.log; exit 1; }
tail -1 ../gpurun_out/r6j_gb_gen.log | cut -c1-900
timeout -k 10 400 python3 -u groupby.py --steps 3 --warmup 1 --source host > ../gpurun_out/r6j_gb_host.log 2>&1 || { tail -20 ../gpurun_out/r6j_gb_host.log; exit 1; }
tail -1 ../gpurun_out/r6j_gb_host.log | cut -c1-900
timeout -k 10 400 python3 -u groupby.py --steps 3 --warmup 1 --source partfile --records-per-gpu 5e8 > ../gpurun_out/r6j_gb_pf.log 2>&1 || { tail -20 ../gpurun_out/r6j_gb_pf.log; exit 1; }
tail -1 ../gpurun_out/r6j_gb_pf.log | cut -c1-900
rm -f /tmp/dryad_groupby_src.pt*
