#!/bin/bash
# GroupBy benchmark under the radix-aggregation and sort paths (name::args per config; the path is
# the GroupByAggregation context property, --aggregation).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_radixagg.py > gpurun_out/ra_t.log 2>&1 || { tail -30 gpurun_out/ra_t.log; exit 1; }
tail -1 gpurun_out/ra_t.log
cd benchmarks
CFGS=("auto::" "radix::--aggregation radix" "sort::--aggregation sort" "radix_wide::--keys 4e18"
      "sort_wide::--aggregation sort --keys 4e18" "radix_k24::--aggregation radix --keys 16777216"
      "sort_k24::--aggregation sort --keys 16777216")
for cfg in "${CFGS[@]}"; do
  [ -n "$GB_ONLY" ] && [[ " $GB_ONLY " != *" ${cfg%%:*} "* ]] && continue
  name=${cfg%%:*}; rest=${cfg#*:}; envs=${rest%%:*}; args=${rest#*:}
  timeout -k 10 300 python -u groupby.py --steps 2 $args > ../gpurun_out/gbc_$name.log 2>&1 || { tail -5 ../gpurun_out/gbc_$name.log; exit 1; }
  echo "$name $(tail -1 ../gpurun_out/gbc_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["validated"])')"
done
