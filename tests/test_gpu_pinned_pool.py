"""Pooled page-locked host buffers (ops/_lib.pinned_lease): a lease released while its copy to
HBM is still queued (a spilled piece read back, runtime/stream_agg.HostPiece) must not be unlocked
or handed to another lease before that copy has run."""
import pytest
import torch

from dryad_amd.ops import _lib

pytestmark = pytest.mark.gpu


def test_released_lease_waits_for_its_queued_copy(monkeypatch):
    monkeypatch.setattr(_lib, "PINNED_KEEP", 0)
    monkeypatch.setattr(_lib, "PINNED_KEEP_BYTES", 0)      # every release evicts (unlocks) at once
    n = 64 << 20
    ls = _lib.pinned_lease((n,), torch.int32)
    ls.tensor.copy_(torch.arange(n, dtype=torch.int32))
    dev = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(4):                                     # queued copies, then the release at once
        dev.copy_(ls.tensor, non_blocking=True)
    buf = ls._buf
    ls.release()
    assert not buf.registered and buf.pending is None      # unlocked only after its copies ran
    torch.cuda.synchronize()
    assert torch.equal(dev[-5:].cpu(), torch.arange(n - 5, n, dtype=torch.int32))


def test_reused_buffer_waits_for_the_previous_lease():
    a = _lib.pinned_lease((1 << 20,), torch.int64)
    a.tensor.fill_(7)
    d = torch.empty(1 << 20, dtype=torch.int64, device="cuda")
    d.copy_(a.tensor, non_blocking=True)
    buf = a._buf
    a.release()
    assert buf.pending is not None or not buf.registered
    b = _lib.pinned_lease((1 << 20,), torch.int64)        # the same buffer: waits for the copy first
    assert b._buf.pending is None
    b.tensor.fill_(9)
    torch.cuda.synchronize()
    assert int(d.sum().item()) == 7 * (1 << 20)
    b.release()
