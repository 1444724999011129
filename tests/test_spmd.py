"""Multi-process SPMD execution of the GPU executor's distributed path on CPU (gloo, 2 ranks)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("ranks,parts", [(2, 2), (2, 3)])
def test_spmd_gloo(ranks, parts):
    env = dict(os.environ, SPMD_DEVICE="cpu", SPMD_PARTS=str(parts), PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist", "spmd_queries.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "SPMD_OK" in r.stdout


def test_query_sweep_cpu_two_ranks():
    """The GPU-executor sweep (tests/dist/gpu_query_sweep_ranks.py) on CPU ranks over gloo."""
    env = dict(os.environ, SPMD_DEVICE="cpu", DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist", "gpu_query_sweep_ranks.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "SWEEP_OK 2" in r.stdout


@pytest.mark.parametrize("ranks", [2, 4])
def test_exchange_gloo(ranks):
    """Device-channel exchange (parallel/exchange.py) of every table layout over gloo ranks."""
    env = dict(os.environ, SPMD_DEVICE="cpu", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist", "exchange_ranks.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"EXCHANGE_OK {ranks}" in r.stdout


@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_chunked_alltoallv_gloo(ranks):
    """The chunked batch_isend_irecv rounds of shuffle.alltoallv_bytes (pairs above the chunk
    size) and the count exchange, byte-exact, over 2, 4 and 8 gloo ranks."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist", "chunked_alltoall_ranks.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"CHUNKED_OK {ranks}" in r.stdout


@pytest.mark.parametrize("ranks", [1, 2])
def test_gpu_executor_fault_kinds_gloo(ranks):
    """Every fault kind (fail, read_error, crash, slow) on the SPMD GPU executor's stage machinery
    (CPU ranks over gloo): oracle-equal results and the expected recovery mechanism."""
    env = dict(os.environ, SPMD_DEVICE="cpu", DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist", "gpu_faults_ranks.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"FAULTS_OK {ranks}" in r.stdout


def test_numa_affinity_helpers(tmp_path):
    """GPU -> NUMA node -> CPU list from a fake sysfs tree (parallel/affinity.py)."""
    from dryad_amd.parallel import affinity as A
    dev = tmp_path / "bus" / "pci" / "devices" / "0000:c1:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text("1\n")
    node = tmp_path / "devices" / "system" / "node" / "node1"
    node.mkdir(parents=True)
    (node / "cpulist").write_text("48-51,96,98-99\n")
    assert A.parse_cpulist("0-2,5,7-8") == {0, 1, 2, 5, 7, 8}
    assert A.gpu_numa_node("0000:C1:00.0", str(tmp_path)) == 1
    assert A.node_cpus(1, str(tmp_path)) == {48, 49, 50, 51, 96, 98, 99}
    (dev / "numa_node").write_text("-1\n")
    assert A.gpu_numa_node("0000:c1:00.0", str(tmp_path)) is None


def test_channel_registry_order_and_registration():
    from dryad_amd.parallel import channels as CHN
    names = [t.name for t in CHN.transports()]
    assert names[:1] == ["device"] and names[-1] == "object"

    class Probe(CHN.Transport):
        name = "probe"

        def usable(self, sends):
            return False

    CHN.register_transport(Probe())
    try:
        assert [t.name for t in CHN.transports()][0] == "probe"
    finally:
        CHN.unregister_transport("probe")
    assert "probe" not in [t.name for t in CHN.transports()]


def test_numa_pci_address_format():
    from types import SimpleNamespace
    from dryad_amd.parallel import affinity as A
    assert A.pci_address(SimpleNamespace(pci_bus_id=0xc1, pci_device_id=0, pci_domain_id=0)) == "0000:c1:00.0"
    assert A.pci_address(SimpleNamespace(pci_bus_id="0000:05:00.0")) == "0000:05:00.0"


@pytest.mark.parametrize("ranks", [2, 3])
def test_size_aware_placement_gloo(ranks, tmp_path):
    """More partitions than ranks over a skewed partfile: partitions are placed by part size
    (largest first on the least-loaded rank) and the results still equal the oracle."""
    env = dict(os.environ, SPMD_DEVICE="cpu", DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT,
               PLACEMENT_DIR=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist", "placement_ranks.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"PLACEMENT_OK {ranks}" in r.stdout
