mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kmeans.py -x -q > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
for d in 0 1; do DRYAD_KM_DEBUG=$d timeout -k 10 100 python tools/microbench_kmeans.py 20000000 16,64,128,256,1024 2>/dev/null | sed "s/^/dbg=$d /" || exit 1; done
