#!/bin/bash
# PMC passes over the TeraSort kernels (one counter group per rocprofv3 run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
N=${N:-400000000}
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "${REGEX:-gather|scatter|count|ts_gen}" \
    -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 \
    --records-per-gpu $N --no-validate > gpurun_out/pmc/p$i.log 2>&1 || { tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
echo PMC_DONE
