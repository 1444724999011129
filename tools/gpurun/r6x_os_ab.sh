#!/bin/bash
# look-back scatter workgroup shape A/B (tools/micro/onesweep_shape_ab.py): in-tree (256 threads x 32
# entries) vs -DDR_OS_SHAPE variants (sort.hip: 2 = 1024 x 16, 4 = 768 x 20, 5 = 1024 x 12; DR_OS_LB look-back depth)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6x
for lib in in-tree $(ls tools/micro/_os_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6x/prof_$tag -o run --output-format csv -- \
    python3 tools/micro/onesweep_shape_ab.py > gpurun_out/r6x/$tag.log 2>&1 || { tail -20 gpurun_out/r6x/$tag.log; exit 1; }
  echo "== $tag: $(grep VALID gpurun_out/r6x/$tag.log)"
  grep "os_scatter" gpurun_out/r6x/prof_$tag/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-60,140-
done
