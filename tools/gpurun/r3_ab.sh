#!/bin/bash
# A/B of the headline bench on one box: round-2 tree (r02tree/) vs the current tree.
set -o pipefail
mkdir -p gpurun_out
for t in cur r02 cur r02; do
  if [ $t = r02 ]; then d=r02tree; else d=.; fi
  (cd $d && timeout -k 10 300 python -u bench.py --steps 10 --warmup 2) > gpurun_out/ab_$t.log 2>&1 || { tail -20 gpurun_out/ab_$t.log; exit 1; }
  echo "$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$t.log) $(grep -o 'OrderBy+Output[^}]*' gpurun_out/ab_$t.log)"
done
