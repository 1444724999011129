"""Two GPU ranks sharing one MI355X (gloo transport staged through the host): exercises the
multi-rank GPU code paths (fused distributed OrderBy, cross shuffles of device tables) that the
8-GPU RCCL run uses, on a single-GPU box."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dump(name, out):
    """Full output of a failed multi-rank run under gpurun_out/ (the assertion shows only a tail)."""
    if out.returncode != 0:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"fail_{name}.log"), "w") as f:
            f.write(out.stdout + "\n---- stderr ----\n" + out.stderr)


@pytest.mark.timeout(600)
def test_two_ranks_share_one_gpu():
    env = dict(os.environ, DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT, TS_RECORDS="2000000")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", "29633",
                          os.path.join(ROOT, "tests", "dist", "gpu_terasort_ranks.py")],
                         capture_output=True, text=True, timeout=560, env=env, cwd=ROOT)
    _dump(os.path.basename(out.args[-1]) + str(len(out.args)), out)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "MULTIRANK_OK 2" in out.stdout


@pytest.mark.timeout(600)
@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_query_sweep_ranks(ranks):
    env = dict(os.environ, DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                          "--master-addr", "127.0.0.1", "--master-port", str(29634 + ranks),
                          os.path.join(ROOT, "tests", "dist", "gpu_query_sweep_ranks.py")],
                         capture_output=True, text=True, timeout=560, env=env, cwd=ROOT)
    _dump(os.path.basename(out.args[-1]) + str(len(out.args)), out)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert f"SWEEP_OK {ranks}" in out.stdout


@pytest.mark.timeout(300)
def test_query_sweep_single_rank():
    """The same sweep on one rank (no cross-rank transport: the local shuffle paths)."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist", "gpu_query_sweep_ranks.py")],
                         capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    _dump(os.path.basename(out.args[-1]) + str(len(out.args)), out)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "SWEEP_OK 1" in out.stdout


@pytest.mark.timeout(400)
@pytest.mark.parametrize("ranks", [2, 4])
def test_exchange_ranks_share_one_gpu(ranks):
    """parallel/exchange.py with device tables on GPU ranks (gloo staging between the ranks):
    the HIP partition kernel's rank-major ports and every table layout, strings included."""
    env = dict(os.environ, DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT, SPMD_DEVICE="cuda")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                          "--master-addr", "127.0.0.1", "--master-port", str(29660 + ranks),
                          os.path.join(ROOT, "tests", "dist", "exchange_ranks.py")],
                         capture_output=True, text=True, timeout=380, env=env, cwd=ROOT)
    _dump(os.path.basename(out.args[-1]) + str(len(out.args)), out)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert f"EXCHANGE_OK {ranks}" in out.stdout


@pytest.mark.timeout(500)
@pytest.mark.parametrize("ranks", [1, 2])
def test_fault_kinds_on_gpu_ranks(ranks):
    """fail / read_error / crash / slow injected into the GPU executor on GPU ranks (device tables,
    device exchange): oracle-equal results and the expected recovery mechanism."""
    env = dict(os.environ, DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT, SPMD_DEVICE="cuda")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                          "--master-addr", "127.0.0.1", "--master-port", str(29680 + ranks),
                          os.path.join(ROOT, "tests", "dist", "gpu_faults_ranks.py")],
                         capture_output=True, text=True, timeout=480, env=env, cwd=ROOT)
    _dump("faults%d" % ranks, out)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert f"FAULTS_OK {ranks}" in out.stdout


@pytest.mark.timeout(960)
@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_fine_rows_ranks_share_one_gpu(ranks, tmp_path):
    """The fine-bucket exchange over materialised tables (generated at a 128-byte pitch, hbm://,
    partfile://) and the GenFusedShuffle variant, validated; skew past capacity stops every rank
    at the vote within seconds (tests/dist/gpu_fine_rows_ranks.py)."""
    env = dict(os.environ, DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT, FINE_TMP=str(tmp_path),
               TS_RECORDS="1500000" if ranks == 2 else "700000")    # (pooled tables: >= 64 MB)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                          "--master-addr", "127.0.0.1", "--master-port", str(29700 + ranks),
                          os.path.join(ROOT, "tests", "dist", "gpu_fine_rows_ranks.py")],
                         capture_output=True, text=True, timeout=920, env=env, cwd=ROOT)
    _dump(os.path.basename(out.args[-1]) + str(ranks), out)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert f"FINE_ROWS_OK {ranks}" in out.stdout


@pytest.mark.timeout(300)
def test_rccl_one_rank_runs_the_collective_paths():
    """A one-rank RCCL communicator with force_collectives: the RCCL branches of the shuffle
    primitives and of the fine-bucket / E128 distributed OrderBy, against real RCCL."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("DRYAD_DIST_BACKEND", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist", "rccl_one_rank.py")],
                         capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    _dump("rccl_one_rank", out)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "RCCL_ONE_RANK_OK" in out.stdout
