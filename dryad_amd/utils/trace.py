"""Timeline ranges for profilers ("roctx ranges per vertex/kernel").

``with trace.range("stage 3:GroupBy[p0]"):`` pushes a roctx range (torch.cuda.nvtx maps to
roctx on ROCm builds), so ``rocprofv3 --marker-trace`` / a ``--sys-trace`` timeline shows which
Dryad stage / vertex / operator issued each kernel.  Disabled with DRYAD_ROCTX=0; a no-op when
no GPU runtime is present.
"""
from __future__ import annotations

import contextlib
import os

_ENABLED = os.environ.get("DRYAD_ROCTX", "1") != "0"
_NVTX = None


def _nvtx():
    global _NVTX, _ENABLED
    if _NVTX is None:
        try:
            import torch
            if not torch.cuda.is_available():
                raise RuntimeError("no GPU")
            from torch.cuda import nvtx
            nvtx.range_push("dryad")
            nvtx.range_pop()
            _NVTX = nvtx
        except Exception:  # noqa: BLE001
            _ENABLED = False
            _NVTX = False
    return _NVTX


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx/nvtx vocabulary
    nv = _nvtx() if _ENABLED else None
    if nv:
        nv.range_push(name)
        try:
            yield
        finally:
            nv.range_pop()
    else:
        yield


def mark(msg: str):
    nv = _nvtx() if _ENABLED else None
    if nv:
        nv.mark(msg)
