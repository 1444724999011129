#!/bin/bash
# rocprofv3 kernel statistics of the headline bench and the secondary BASELINE benchmarks
# (one run each, kernel trace + stats only).  Each GPU step has its own time limit; the script
# stops at the first failure.  Optional $1: subset "ts", "gb", "km", "join" (default all).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
WHICH=${1:-ts,gb,km,join}
run() {   # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$name -o run -- "$@" \
    > $R/gpurun_out/prof_$name.log 2>&1 || { tail -30 $R/gpurun_out/prof_$name.log; exit 1; }
  tail -1 $R/gpurun_out/prof_$name.log
}
case $WHICH in *ts*) run ts 300 python3 $R/bench.py --steps 3 --warmup 1;; esac
cd $R/benchmarks
case $WHICH in *gb*) run gb 300 python3 groupby.py --steps 3 --warmup 1;; esac
case $WHICH in *km*) run km 300 python3 kmeans.py --iters 3 --warmup 1;; esac
case $WHICH in *join*) run join 400 python3 join.py --steps 1 --warmup 1;; esac
cd $R
for d in gpurun_out/prof_*/; do
  db=$(find $d -name '*.db' | head -1)
  [ -n "$db" ] && python3 tools/rocpd_summary.py "$db" --csv "${d%/}_kernels.csv" > /dev/null
done
ls gpurun_out
