set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gb3 -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/groupby.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/gb_prof.log 2>&1; rc=$?
tail -1 $GRAFT_REPO_ROOT/gpurun_out/gb_prof.log; exit $rc
