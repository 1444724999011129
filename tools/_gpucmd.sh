set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_grace.py -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -15 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/join.py --table-gb 4 --steps 2 --hbm-budget-gb 4 > gpurun_out/join_small_spill.log 2>&1; rc=$?; tail -1 gpurun_out/join_small_spill.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python benchmarks/join.py --steps 2 > gpurun_out/join_full.log 2>&1; rc=$?; tail -2 gpurun_out/join_full.log; exit $rc
