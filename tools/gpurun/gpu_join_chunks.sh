#!/bin/bash
# join benchmark at several producer chunk sizes (a chunk that fits the Infinity Cache keeps the
# generate -> count -> scatter round trip on die).  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
cd benchmarks || exit 1
for c in ${CHUNKS:-2097152 4194304 16777216}; do
  timeout -k 10 300 python -u join.py --steps 3 --warmup 1 --chunk-rows $c > ../gpurun_out/join_c$c.log 2>&1 \
    || { tail -20 ../gpurun_out/join_c$c.log; exit 1; }
  echo "chunk $c: $(tail -1 ../gpurun_out/join_c$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["validated"])')"
done
