"""Per-job operator strategy choices, taken from context properties (no import-time environment
knobs in the kernel library): the GPU executor enters ``scope(ctx)`` for each job on its job
thread, and operators read ``current()``.  Outside a job the defaults apply.

    GroupByAggregation   "auto" | "radix" | "sort": radix-partitioned LDS aggregation for a
                         single integer key (ops/radixagg.py) only for keys spanning >= 2^32
                         values ("auto"), for every large integer key ("radix"), or never ("sort").
"""
from __future__ import annotations

import contextlib
import contextvars
from dataclasses import dataclass, replace


@dataclass(frozen=True)
class Tuning:
    groupby_aggregation: str = "auto"


_CUR: contextvars.ContextVar = contextvars.ContextVar("dryad_tuning", default=Tuning())


def current() -> Tuning:
    return _CUR.get()


def from_ctx(ctx) -> Tuning:
    props = ctx._props if ctx is not None else {}
    agg = props.get("GroupByAggregation") or "auto"
    if agg not in ("auto", "radix", "sort"):
        raise ValueError(f"GroupByAggregation must be auto, radix or sort, not {agg!r}")
    return replace(Tuning(), groupby_aggregation=agg)


@contextlib.contextmanager
def scope(ctx=None, **kw):
    t = replace(from_ctx(ctx), **kw) if ctx is not None else replace(current(), **kw)
    tok = _CUR.set(t)
    try:
        yield t
    finally:
        _CUR.reset(tok)
