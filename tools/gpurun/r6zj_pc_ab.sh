#!/bin/bash
# row-staged channel scatter (channel.hip pc_scatter_rows_kernel) workgroup A/B: in-tree 256 threads x
# 512-row tiles vs -DDR_PC_ROWS_NT variants (tile = 2 x threads); channel / stream-shuffle GPU tests
# per library, then the 8-rank GroupBy per-rank program (streamed shuffle) under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zj
for lib in in-tree $(ls tools/micro/_pc_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 400 python -u -m pytest tests/test_gpu_channel.py tests/test_gpu_stream_shuffle.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r6zj/$tag.tests.log 2>&1 || { tail -30 gpurun_out/r6zj/$tag.tests.log; exit 1; }
  echo "== $tag: $(tail -1 gpurun_out/r6zj/$tag.tests.log)"
  (cd benchmarks && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d ../gpurun_out/r6zj/prof_$tag -o run --output-format csv -- \
    python3 groupby.py --loopback-ranks 8 --steps 2 --warmup 1 --stream-shuffle --hbm-budget-gb 200 > ../gpurun_out/r6zj/$tag.log 2>&1) \
    || { tail -20 gpurun_out/r6zj/$tag.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"ok": [a-z]*\|"stage_a_ms": [0-9.]*' gpurun_out/r6zj/$tag.log | tr '\n' ' '; echo
  grep "pc_scatter_rows" gpurun_out/r6zj/prof_$tag/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-45,100-
done
