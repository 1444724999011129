#!/bin/bash
# GroupBy segmented-reduction input layouts: tests, then the benchmark A/B (columns vs packed rows)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_ops.py tests/test_gpu_executor.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/gpu_t3.log 2>&1 || { tail -40 gpurun_out/gpu_t3.log; exit 1; }
tail -2 gpurun_out/gpu_t3.log
cd benchmarks || exit 1
timeout -k 10 300 python -u groupby.py --steps 3 --warmup 1 > ../gpurun_out/gb_aos.log 2>&1 || { tail -20 ../gpurun_out/gb_aos.log; exit 1; }
tail -1 ../gpurun_out/gb_aos.log
DRYAD_SEGRED_AOS_MIN_ROWS=4611686018427387904 timeout -k 10 300 python -u groupby.py --steps 3 --warmup 1 \
  > ../gpurun_out/gb_cols.log 2>&1 || { tail -20 ../gpurun_out/gb_cols.log; exit 1; }
tail -1 ../gpurun_out/gb_cols.log
cd .. || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gbaos -o gb -- python3 benchmarks/groupby.py --steps 2 --warmup 1 \
  > gpurun_out/gb_prof.log 2>&1 || { tail -20 gpurun_out/gb_prof.log; exit 1; }
echo prof done
