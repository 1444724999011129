#!/bin/bash
# end-of-round check after the channel / dense-group grid changes: GPU suite, smoke, 1-GPU bench,
# GroupBy 1-GPU and 8-rank loopback (unprofiled)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c_final2_suite.log 2>&1 || { tail -40 gpurun_out/r5c_final2_suite.log; exit 1; }
tail -1 gpurun_out/r5c_final2_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5c_final2_smoke.log 2>&1 || { tail -20 gpurun_out/r5c_final2_smoke.log; exit 1; }
tail -1 gpurun_out/r5c_final2_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5c_final2_bench.log 2>&1 || { tail -20 gpurun_out/r5c_final2_bench.log; exit 1; }
tail -1 gpurun_out/r5c_final2_bench.log | cut -c1-300
cd benchmarks
timeout -k 10 300 python3 -u groupby.py --steps 5 --warmup 1 > ../gpurun_out/r5c_final2_gb.log 2>&1 || { tail -20 ../gpurun_out/r5c_final2_gb.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"validated": [a-z]*' ../gpurun_out/r5c_final2_gb.log | tr '\n' ' '; echo
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 4 --warmup 1 > ../gpurun_out/r5c_final2_gblb8.log 2>&1 || { tail -20 ../gpurun_out/r5c_final2_gblb8.log; exit 1; }
grep "step\|warmup" ../gpurun_out/r5c_final2_gblb8.log | cut -c1-120
grep -o '"ms_per_step": [0-9.]*\|"validated": {"ok": [a-z]*' ../gpurun_out/r5c_final2_gblb8.log | tr '\n' ' '; echo
