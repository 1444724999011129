set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_executor.py tests/test_gpu_kmeans.py -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/kmeans.py --iters 5 > gpurun_out/km_bench.log 2>&1; rc=$?; tail -3 gpurun_out/km_bench.log; exit $rc
