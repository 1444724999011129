set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_executor.py -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -30 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/groupby.py --steps 2 --keys 1000 > gpurun_out/gb_1k.log 2>&1; rc=$?; tail -1 gpurun_out/gb_1k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/groupby.py --steps 2 > gpurun_out/gb_full.log 2>&1; rc=$?; tail -1 gpurun_out/gb_full.log; exit $rc
