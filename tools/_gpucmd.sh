set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1; rc=$?
grep metric $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log; exit $rc
