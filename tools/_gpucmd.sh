set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_sort.py tests/test_gpu_executor.py tests/test_gpu_kmeans.py -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -25 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for d in 0 1; do DRYAD_KM_DEBUG=$d timeout -k 10 100 python tools/microbench_kmeans.py 20000000 16,64,128,256,1024 2>/dev/null | sed "s/^/dbg=$d /" || exit 1; done
timeout -k 10 600 python benchmarks/groupby.py --steps 2 > gpurun_out/gb_full.log 2>&1; rc=$?; tail -1 gpurun_out/gb_full.log; exit $rc
