#!/bin/bash
# host profile of the stored-data TeraSort steps (where the ~0.3 s beyond read + sort + write go)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m cProfile -o gpurun_out/stored.prof bench.py --records-per-gpu 250000000 --input partfile:///tmp/ts_in \
  --output partfile:///tmp/ts_out --steps 4 --warmup 1 --no-validate > gpurun_out/r5b_stored_prof.log 2>&1 || { tail -20 gpurun_out/r5b_stored_prof.log; exit 1; }
grep '"metric"' gpurun_out/r5b_stored_prof.log | cut -c1-200
python3 -c "
import pstats
p = pstats.Stats('gpurun_out/stored.prof')
p.sort_stats('cumulative').print_stats(45)
" > gpurun_out/r5b_stored_pstats.txt 2>&1
head -120 gpurun_out/r5b_stored_pstats.txt | cut -c1-180
