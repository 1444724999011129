#!/bin/bash
# dense GroupBy aggregation workgroup A/B (-DDR_DG_AGG_NT threads, -DDR_DG_AGG_U rows per thread per step) vs
# the in-tree 512 x 4: densegroup numerics per variant, then the 1-GPU GroupBy bench under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in in-tree $(ls tools/micro/_dg_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_densegroup.py -q --timeout 120 --timeout-method thread \
    > gpurun_out/r6zc_dgab_$tag.tests.log 2>&1 || { tail -30 gpurun_out/r6zc_dgab_$tag.tests.log; exit 1; }
  (cd benchmarks && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_r6zc_dgab_$tag -o run --output-format csv -- \
    python3 groupby.py --steps 3 --warmup 1 > ../gpurun_out/r6zc_dgab_$tag.log 2>&1) || { tail -20 gpurun_out/r6zc_dgab_$tag.log; exit 1; }
  echo "== $tag: $(tail -1 gpurun_out/r6zc_dgab_$tag.tests.log)"
  grep -o '"ms_per_step": [0-9.]*\|"validated": [a-z]*' gpurun_out/r6zc_dgab_$tag.log | tr '\n' ' '; echo
  grep "dg_agg" gpurun_out/prof_r6zc_dgab_$tag/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-50,120-
done
