#!/bin/bash
# GroupBy benchmark A/B (AoS-packed segmented reduction on / off) + kernel statistics
set -o pipefail
mkdir -p gpurun_out
cd benchmarks || exit 1
timeout -k 10 300 python -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/gb_aos.log 2>&1 || { tail -20 ../gpurun_out/gb_aos.log; exit 1; }
tail -1 ../gpurun_out/gb_aos.log
DRYAD_SEGRED_AOS_MIN_ROWS=4611686018427387904 timeout -k 10 300 python -u groupby.py --steps 3 --warmup 1 \
  > ../gpurun_out/gb_noaos.log 2>&1 || { tail -20 ../gpurun_out/gb_noaos.log; exit 1; }
tail -1 ../gpurun_out/gb_noaos.log
cd .. || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gb -o gb -- python3 benchmarks/groupby.py --steps 2 --warmup 1 \
  > gpurun_out/gb_prof.log 2>&1 || { tail -20 gpurun_out/gb_prof.log; exit 1; }
find gpurun_out/prof_gb -name "*.db" | head -3
