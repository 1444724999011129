#!/bin/bash
# partition-channel grid cap variants (tools/micro/_pc_ab, -DDR_PC_GMAX) against the in-tree library:
# channel numerics per variant, then the 8-rank GroupBy loopback (row scatter per call) under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in in-tree $(ls tools/micro/_pc_ab/*.so); do
  tag=$(basename $lib .so)
  if [ $lib = in-tree ]; then unset DRYAD_KERNEL_LIB; else export DRYAD_KERNEL_LIB=$PWD/$lib; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_channel.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r5c_pcab_$tag.tests.log 2>&1 || { tail -30 gpurun_out/r5c_pcab_$tag.tests.log; exit 1; }
  (cd benchmarks && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_pcab_$tag -o run --output-format csv -- \
    python3 -u groupby.py --loopback-ranks 8 --steps 2 --warmup 1 > ../gpurun_out/r5c_pcab_$tag.log 2>&1) || { tail -20 gpurun_out/r5c_pcab_$tag.log; exit 1; }
  echo "== $tag: $(tail -1 gpurun_out/r5c_pcab_$tag.tests.log)"
  grep -o '"ms_per_step": [0-9.]*\|"validated": {"ok": [a-z]*' gpurun_out/r5c_pcab_$tag.log | tr '\n' ' '; echo
done
