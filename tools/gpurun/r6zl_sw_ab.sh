#!/bin/bash
# wide-entry (E256 / E320) sort pass A/B (tools/micro/sortwide_ab.py through relational.payload_groups):
# in-tree rs_scatter_v2 (256 threads) vs rs_scatter_w variants (-DDR_SORTW_*), validated vs torch;
# device-op GPU tests per library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zl
for lib in in-tree $(ls tools/micro/_sw_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6zl/prof_$tag -o run --output-format csv -- \
    python3 tools/micro/sortwide_ab.py > gpurun_out/r6zl/$tag.log 2>&1 || { tail -20 gpurun_out/r6zl/$tag.log; exit 1; }
  echo "== $tag: $(grep VALID gpurun_out/r6zl/$tag.log)"
  grep "rs_scatter" gpurun_out/r6zl/prof_$tag/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-45,100-
  rm -f gpurun_out/r6zl/prof_$tag/run_kernel_trace.csv
  timeout -k 10 300 python -u -m pytest tests/test_gpu_device_ops.py tests/test_gpu_sort.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r6zl/$tag.tests.log 2>&1 || { tail -30 gpurun_out/r6zl/$tag.tests.log; exit 1; }
  echo "   tests: $(tail -1 gpurun_out/r6zl/$tag.tests.log)"
done
