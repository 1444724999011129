set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_executor.py -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/groupby.py --records-per-gpu 1e8 --steps 2 > gpurun_out/gb_small.log 2>&1; rc=$?; tail -2 gpurun_out/gb_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/groupby.py --steps 2 > gpurun_out/gb_full.log 2>&1; rc=$?; tail -2 gpurun_out/gb_full.log; exit $rc
