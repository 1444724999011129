"""Calling ``@device_function`` Apply bodies from any executor.

The GPU executor passes its HBM ``DeviceTable`` partitions straight through; LocalDebug and the
CPU executors hold records, so the records are turned into CPU-tensor tables first (using the
plan's input dtypes) and the returned table back into records.  One user function therefore has
one meaning everywhere, and the LocalDebug oracle can check the GPU result.
"""
from __future__ import annotations


def to_table(x, dtype, device):
    from .gpu.table import DeviceTable, from_objects
    if isinstance(x, DeviceTable):
        return x if str(x.device) == str(device) else _move(x, device)
    t = from_objects(list(x), dtype, device)
    if t is None:
        raise TypeError(f"device_function input of type {dtype!r} is not columnar")
    return t


def _move(t, device):
    from .gpu.table import DeviceTable
    if t.rows is not None:
        return DeviceTable(t.n, t.shape, rows=t.rows.to(device))
    return DeviceTable(t.n, t.shape, {k: v.to(device) for k, v in t.cols.items()})


def call(fn, inputs: list, in_dtypes: list, multi: bool, device="cpu"):
    """Run ``fn`` on table versions of ``inputs``; returns whatever ``fn`` returns."""
    dts = list(in_dtypes or []) + [None] * (len(inputs) - len(in_dtypes or []))
    tables = [to_table(x, dt, device) for x, dt in zip(inputs, dts)]
    return fn(tables) if multi else fn(*tables)


def call_on_records(fn, inputs: list, in_dtypes: list, multi: bool) -> list:
    from .gpu.table import DeviceTable
    res = call(fn, inputs, in_dtypes, multi, "cpu")
    if isinstance(res, DeviceTable):
        return res.to_objects()
    return list(res)
