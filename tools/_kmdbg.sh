#!/bin/bash
# k-means kernel phase costs: DRYAD_KM_DEBUG bit0 skips the sum MFMAs, bit1 the distance MFMAs,
# bit2 the near-tie re-rank, bit3 counts the re-ranked points.
set -o pipefail
mkdir -p gpurun_out
for d in 8 0 4 1 6 7; do
  DRYAD_KM_DEBUG=$d timeout -k 10 120 python -u tools/microbench_kmeans.py 125e6 64 > gpurun_out/kmdbg_$d.log 2>&1 || { tail -5 gpurun_out/kmdbg_$d.log; exit 1; }
  echo "dbg=$d $(grep -h 'near-tie' gpurun_out/kmdbg_$d.log | tail -1) $(tail -1 gpurun_out/kmdbg_$d.log)"
done
