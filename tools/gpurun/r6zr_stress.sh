#!/bin/bash
# exactness stress of the count-matrix sorts over many sizes: in-tree kernels and the 16-wave variant
# library (every DR_SORT*_NT switch on)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zr
for lib in in-tree tools/micro/_stress/libsort_wide_all.so; do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u tools/micro/sort_stress.py > gpurun_out/r6zr/$tag.log 2>&1 || { tail -20 gpurun_out/r6zr/$tag.log; exit 1; }
  echo "== $tag: $(grep STRESS gpurun_out/r6zr/$tag.log)"
done
