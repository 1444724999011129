#!/bin/bash
# round 6: after the 1024 x 16 look-back scatter and the 8192-row dense GroupBy tiles: sort / TeraSort /
# GroupBy GPU tests, then bench.py (TeraSort 125 GB) and the GroupBy bench with kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6z
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sort.py \
  tests/test_gpu_compact_sort.py tests/test_gpu_fine_rows.py tests/test_gpu_pitch128.py tests/test_gpu_tsmerge.py \
  tests/test_gpu_densegroup.py tests/test_gpu_extsort.py tests/test_gpu_rowpack.py > gpurun_out/r6z/tests.log 2>&1 \
  || { tail -30 gpurun_out/r6z/tests.log; exit 1; }
tail -1 gpurun_out/r6z/tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6z/bench.log 2>&1 || { tail -20 gpurun_out/r6z/bench.log; exit 1; }
grep '"metric"' gpurun_out/r6z/bench.log | cut -c1-400
(cd benchmarks && timeout -k 10 300 python -u groupby.py > ../gpurun_out/r6z/groupby.log 2>&1) || { tail -20 gpurun_out/r6z/groupby.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"validated": [a-z]*' gpurun_out/r6z/groupby.log | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6z/ts_prof -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 > gpurun_out/r6z/bench_prof.log 2>&1 || { tail -20 gpurun_out/r6z/bench_prof.log; exit 1; }
echo done
