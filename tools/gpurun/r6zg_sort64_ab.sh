#!/bin/bash
# E64 count + scatter sort pass shape A/B (tools/micro/onesweep_shape_ab.py ... count): in-tree
# rs_scatter_v3 (256 x 16) vs rs_scatter_w (-DDR_SORT64_NT); the in-tree E128 sort (now 1024 x 8);
# the sort GPU tests per library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zg
timeout -k 10 240 python3 tools/micro/sort128_shape_ab.py > gpurun_out/r6zg/sort128_in-tree.log 2>&1 || { tail -20 gpurun_out/r6zg/sort128_in-tree.log; exit 1; }
echo "== E128 in-tree: $(grep VALID gpurun_out/r6zg/sort128_in-tree.log)"
for lib in in-tree $(ls tools/micro/_sort_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6zg/prof_$tag -o run --output-format csv -- \
    python3 tools/micro/onesweep_shape_ab.py 1.25e9 count > gpurun_out/r6zg/$tag.log 2>&1 || { tail -20 gpurun_out/r6zg/$tag.log; exit 1; }
  echo "== $tag: $(grep VALID gpurun_out/r6zg/$tag.log)"
  grep "rs_scatter" gpurun_out/r6zg/prof_$tag/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-50,100-
  timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_device_ops.py tests/test_gpu_compact_sort.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r6zg/$tag.tests.log 2>&1 || { tail -30 gpurun_out/r6zg/$tag.tests.log; exit 1; }
  echo "   tests: $(tail -1 gpurun_out/r6zg/$tag.tests.log)"
done
