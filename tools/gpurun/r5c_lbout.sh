#!/bin/bash
# GroupBy loopback after the 1-GPU GroupBy (the order in which a 1.8 s stage B step appeared):
# the previous step's output released at the start of each step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/benchmarks" || exit 1
mkdir -p ../gpurun_out
timeout -k 10 300 python3 -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/r5c_lbout_gb.log 2>&1 || { tail -20 ../gpurun_out/r5c_lbout_gb.log; exit 1; }
grep -o '"value": [0-9.]*\|"validated": [a-z]*' ../gpurun_out/r5c_lbout_gb.log | tr '\n' ' '; echo
timeout -k 10 500 python3 -u groupby.py --loopback-ranks 8 --steps 6 --warmup 1 > ../gpurun_out/r5c_lbout_gblb8.log 2>&1 || { tail -20 ../gpurun_out/r5c_lbout_gblb8.log; exit 1; }
grep "step\|warmup" ../gpurun_out/r5c_lbout_gblb8.log | cut -c1-120
grep -o '"ms_per_step": [0-9.]*\|"validated": {"ok": [a-z]*\|"hbm_[a-z_]*GB": [0-9.]*' ../gpurun_out/r5c_lbout_gblb8.log | tr '\n' ' '; echo
