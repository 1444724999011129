#!/bin/bash
# E128 count-matrix sort pass shape A/B (tools/micro/sort128_shape_ab.py): in-tree rs_scatter_v2 (256
# threads x 8) vs rs_scatter_w variants; validated sort + kernel stats; then the sort GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zf
for lib in in-tree $(ls tools/micro/_sort_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6zf/prof_$tag -o run --output-format csv -- \
    python3 tools/micro/sort128_shape_ab.py > gpurun_out/r6zf/$tag.log 2>&1 || { tail -20 gpurun_out/r6zf/$tag.log; exit 1; }
  echo "== $tag: $(grep VALID gpurun_out/r6zf/$tag.log)"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_device_ops.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r6zf/$tag.tests.log 2>&1 || { tail -30 gpurun_out/r6zf/$tag.tests.log; exit 1; }
  echo "   tests: $(tail -1 gpurun_out/r6zf/$tag.tests.log)"
done
