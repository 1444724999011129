set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_gb -o run -- python3 $R/benchmarks/groupby.py --steps 1 --warmup 1 > $R/gpurun_out/p_gb.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_gb1k -o run -- python3 $R/benchmarks/groupby.py --steps 1 --warmup 1 --keys 1000 > $R/gpurun_out/p_gb1k.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_km -o run -- python3 $R/benchmarks/kmeans.py --iters 3 --warmup 1 > $R/gpurun_out/p_km.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_join -o run -- python3 $R/benchmarks/join.py --steps 1 --warmup 1 > $R/gpurun_out/p_join.log 2>&1 || exit 1
grep -h metric $R/gpurun_out/p_*.log | cut -c1-200
