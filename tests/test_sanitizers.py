"""Host-side sanitizer runs of the native runtime: the job graph, codec, text
splitting, WorkQueue and ChunkReader self-test built with -fsanitize=address,undefined and with
-fsanitize=thread.  (GPU sanitizers are not available on this pool; kernels are covered by the
numerics tests.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "runtime", f) for f in ("jobgraph.cpp", "codec.cpp", "workqueue.cpp", "partreader.cpp")]
TEST = os.path.join(ROOT, "csrc", "runtime", "tests", "selftest.cpp")


def _build_and_run(tmp_path, flags, env=None):
    cxx = os.environ.get("CXX", "g++")
    if shutil.which(cxx) is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "selftest")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-I", os.path.join(ROOT, "csrc", "runtime"),
           *SRC, TEST, "-o", exe, "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=240)
    out = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=240,
                         env=dict(os.environ, **(env or {})))
    assert out.returncode == 0, out.stdout + out.stderr
    assert "SELFTEST_OK" in out.stdout


@pytest.mark.timeout(600)
def test_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})


@pytest.mark.timeout(600)
def test_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
