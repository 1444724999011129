"""Column value bounds (min / max) of device columns, cached per tensor.

Operators that pack rows by value width (ops/densegroup.py) need bounds, not exact extremes:
lo <= every value <= hi.  Sources that know them for free register them when they build a column
(the gen:// generators: a key column over [0, keys), 31-bit payloads), the way a columnar file
format keeps per-column statistics in its footer; any other column gets one fused min/max pass
(ops/reduce.reduce_multi, up to 8 columns per pass) the first time it is asked for.  An entry dies
with its tensor and is ignored once the tensor has been modified in place.
"""
from __future__ import annotations

import torch
from torch.utils.weak import WeakIdKeyDictionary

_BOUNDS = WeakIdKeyDictionary()


def set_bounds(col: torch.Tensor, lo: int, hi: int) -> None:
    """Declare lo <= col[i] <= hi for every row (integer columns)."""
    _BOUNDS[col] = (int(lo), int(hi), col._version)


def known(col: torch.Tensor):
    e = _BOUNDS.get(col)
    if e is None or e[2] != col._version:
        return None
    return e[0], e[1]


def inherit(dst: torch.Tensor, src: torch.Tensor) -> None:
    """``dst`` holds a subset (or a copy) of ``src``'s values: it keeps src's bounds."""
    b = known(src)
    if b is not None:
        set_bounds(dst, *b)


def union(dst: torch.Tensor, srcs: list) -> None:
    """``dst`` holds the values of ``srcs`` (concatenated): bounds when every source has them."""
    bs = [known(x) for x in srcs]
    if bs and all(b is not None for b in bs):
        set_bounds(dst, min(b[0] for b in bs), max(b[1] for b in bs))


def bounds(cols: list) -> list:
    """[(lo, hi)] for integer columns (one device pass over those without registered bounds)."""
    out = [known(c) for c in cols]
    missing = [i for i, b in enumerate(out) if b is None]
    if missing:
        from ..ops import reduce as RD
        n = cols[missing[0]].shape[0]
        slots = []
        for i in missing:
            c = cols[i] if cols[i].dtype == torch.int64 else cols[i].to(torch.int64)
            slots += [(RD.MIN, c, None), (RD.MAX, c, None)]
        got = RD.reduce_multi(n, slots, cols[missing[0]].device)
        for j, i in enumerate(missing):
            out[i] = (int(got[2 * j]), int(got[2 * j + 1]))
            set_bounds(cols[i], *out[i])
    return out


class BoundsAcc:
    """Union of the integer columns' [min, max] over the pieces of a table written piece by piece
    (a stored table keeps them in its schema, runtime/gpu_executor._commit_partfile_impl).
    ``result()`` is None once a piece was not a columnar device table (nothing known then)."""

    _INT = (torch.int64, torch.int32, torch.int16, torch.int8)

    def __init__(self):
        self.bounds, self.ok = {}, True

    def add(self, t) -> None:
        if not self.ok:
            return
        cols = getattr(t, "cols", None)
        if cols is None or getattr(t, "rows", None) is not None or getattr(t, "strs", None):
            if getattr(t, "n", len(t) if isinstance(t, list) else 1):
                self.ok = False
            return
        if t.n == 0:
            return
        for f, c in cols.items():
            if c.dtype not in self._INT:
                continue
            kb = known(c)
            if kb is None:
                mn, mx = torch.aminmax(c[: t.n])
                kb = (int(mn.item()), int(mx.item()))
            o = self.bounds.get(f)
            self.bounds[f] = [kb[0], kb[1]] if o is None else [min(o[0], kb[0]), max(o[1], kb[1])]

    def result(self):
        return dict(self.bounds) if self.ok else None
