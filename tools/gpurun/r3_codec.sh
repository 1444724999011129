#!/bin/bash
# Variable-length codec / reader tests, reader bandwidth, WordCount over a partfile.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec_var.py tests/test_gpu_channel.py tests/test_gpu_text.py -m gpu -q \
  --timeout 200 --timeout-method thread > gpurun_out/codec_tests.log 2>&1
rc=$?
tail -30 gpurun_out/codec_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/microbench_reader.py 8 > gpurun_out/reader_bench.log 2>&1 || { tail -20 gpurun_out/reader_bench.log; exit 1; }
tail -2 gpurun_out/reader_bench.log
exit $rc
