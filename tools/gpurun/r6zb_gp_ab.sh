#!/bin/bash
# join staged-projection partition scatter (grace.hip gp_scatter_kernel STAGE_PROJ, -DDR_GP_PROJ_NT /
# -DDR_GP_PROJ_ITEMS variant libraries) vs in-tree 256 x 8: grace GPU tests, then the 2 x 100 GB join
# bench under rocprofv3 kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6zb
for lib in in-tree $(ls tools/micro/_gp_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_grace.py tests/test_gpu_grace_stage.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r6zb/$tag.tests.log 2>&1 || { tail -30 gpurun_out/r6zb/$tag.tests.log; exit 1; }
  (cd benchmarks && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/r6zb/prof_$tag -o run \
    --output-format csv -- python3 join.py --steps 2 --warmup 1 > ../gpurun_out/r6zb/$tag.log 2>&1) \
    || { tail -20 gpurun_out/r6zb/$tag.log; exit 1; }
  echo "== $tag: $(tail -1 gpurun_out/r6zb/$tag.tests.log)"
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"validated": [a-z]*' gpurun_out/r6zb/$tag.log | tr '\n' ' '; echo
  grep "gp_scatter\|rp_scatter" gpurun_out/r6zb/prof_$tag/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-50,100-
done
