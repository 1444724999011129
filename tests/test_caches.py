"""Caches keyed on a tensor's version counter must see writes done by native kernels (ADVICE r3:
column bounds and k-means planes went stale when a generator rewrote an existing tensor)."""
import torch

from dryad_amd.gpu import stats
from dryad_amd.ops import _lib


def test_written_invalidates_version_keyed_caches():
    t = torch.arange(10)
    stats.set_bounds(t, 0, 9)
    assert stats.known(t) == (0, 9)
    _lib.written(t)                       # a kernel rewrote t through its pointer
    assert stats.known(t) is None
    stats.set_bounds(t, 0, 9)
    _lib.written(t[2:5])                  # ... or a view of it
    assert stats.known(t) is None
