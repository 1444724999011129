#!/bin/bash
# round 6: overlapped TeraSort exchange, wide grace rows, streamed shuffle / sinks; 8-rank loopback
# with the modelled link; one-rank RCCL at the full 125 GB
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fine_rows.py tests/test_gpu_tsmerge.py tests/test_gpu_multirank.py -x -q --timeout 880 --timeout-method thread > gpurun_out/r6c_tests.log 2>&1 || { tail -60 gpurun_out/r6c_tests.log; exit 1; }
tail -1 gpurun_out/r6c_tests.log
timeout -k 10 400 python -u bench.py --loopback-ranks 8 --steps 3 --warmup 1 > gpurun_out/r6c_lb8.log 2>&1 || { tail -20 gpurun_out/r6c_lb8.log; exit 1; }
grep "step" gpurun_out/r6c_lb8.log | cut -c1-250
tail -1 gpurun_out/r6c_lb8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], c['phases_ms'], c['validated'], c['modelled_exchange'])"
timeout -k 10 400 python -u bench.py --rccl-one-rank --steps 3 --warmup 1 > gpurun_out/r6c_rccl1.log 2>&1 || { tail -20 gpurun_out/r6c_rccl1.log; exit 1; }
tail -1 gpurun_out/r6c_rccl1.log | cut -c1-2500
df -h /dev/shm /tmp | tee gpurun_out/r6c_df.txt
timeout -k 10 300 python -u tools/ckpt_bench.py --gb 25 > gpurun_out/r6c_ckpt.log 2>&1 || { tail -20 gpurun_out/r6c_ckpt.log; exit 1; }
tail -3 gpurun_out/r6c_ckpt.log
