"""``gen://names``: a synthetic table with a string key, for string-keyed joins and GroupBys.

Record i is ``(Name, V1, V2)``: the records64 generator's columns Key, V1, V2 (models/records_cpu.py,
csrc/kernels/generators.hip) with the key rendered as the string ``"u" + decimal(Key)`` (2..20
bytes), so both the host oracle and the device path derive it from the same counter-based
generator.  ``&mode=dim`` makes the keys a bijection of [0, K) (a dimension table).
``&namelen=L`` (L > 20) zero-pads every name to exactly L bytes: "u" + decimal(Key) right-aligned
in L - 1 digits (long string keys for the grace join's out-of-line widening)."""
from __future__ import annotations

import torch

FIELDS = ["Name", "V1", "V2"]


def namelen(q: dict) -> int:
    """The fixed name length of a gen://names query (0: natural "u<decimal>" lengths)."""
    L = int(q.get("namelen", 0) or 0)
    if L and L <= 20:
        raise ValueError("gen://names: namelen must exceed 20 (the longest natural name)")
    return L


def host_records(first: int, n: int, nkeys: int, seed: int, dim_mult: int = 0, name_len: int = 0) -> list:
    from .records_cpu import gen_columns
    k, v1, v2 = gen_columns(first, n, nkeys, seed, 3, dim_mult)
    if name_len:
        return [("u" + str(a).rjust(name_len - 1, "0"), b, c) for a, b, c in zip(k.tolist(), v1.tolist(), v2.tolist())]
    return [("u" + str(a), b, c) for a, b, c in zip(k.tolist(), v1.tolist(), v2.tolist())]


def max_name_bytes(name_len: int = 0) -> int:
    return name_len or 20


def render(keys: torch.Tensor, name_len: int = 0):
    """Non-negative int64 keys -> (heap uint8, offsets int64, lengths int64) of "u<decimal>" on
    the keys' device: digits right-aligned in a 20-byte field, then one boolean-mask compaction
    (row-major) keeps 'u' and the significant digits of each row.  ``name_len``: every name is
    that long ('u', zeros, the digits), the heap is the [n, name_len] buffer itself."""
    n = keys.shape[0]
    dev = keys.device
    if name_len:
        buf = torch.full((n, name_len), ord("0"), dtype=torch.uint8, device=dev)
        buf[:, 0] = ord("u")
        x = keys.clone()
        for j in range(name_len - 1, max(0, name_len - 20), -1):
            buf[:, j] = (x % 10).to(torch.uint8) + ord("0")
            x = torch.div(x, 10, rounding_mode="floor")
        ln = torch.full((n,), name_len, dtype=torch.int64, device=dev)
        return buf.view(-1), torch.arange(n, dtype=torch.int64, device=dev) * name_len, ln
    buf = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    buf[:, 0] = ord("u")
    x = keys.clone()
    nd = torch.ones(n, dtype=torch.int64, device=dev)
    for j in range(19, 0, -1):
        buf[:, j] = (x % 10).to(torch.uint8) + ord("0")
        x = torch.div(x, 10, rounding_mode="floor")
        if j > 1:
            nd += (x > 0).to(torch.int64)
    col = torch.arange(20, device=dev).view(1, 20)
    mask = (col == 0) | (col >= (20 - nd).view(n, 1))
    heap = buf[mask]
    ln = nd + 1
    off = torch.cumsum(ln, 0) - ln
    return heap, off, ln


def device_table(first: int, n: int, nkeys: int, seed: int, dim_mult: int, device, name_len: int = 0):
    """The records first .. first + n - 1 as a columnar DeviceTable with a string Name field."""
    from ..gpu.table import DeviceTable, Shape
    from ..ops import relational as R
    cols = [torch.empty(n, dtype=torch.int64, device=device) for _ in range(3)]
    if n:
        R.gen_records64(cols, first, nkeys, seed, dim_mult)
    heap, off, ln = render(cols[0], name_len)
    return DeviceTable(n, Shape("tuple", list(FIELDS)), {"Name": off, "Name#len": ln, "V1": cols[1], "V2": cols[2]},
                       strs={"Name": heap})


def dtype():
    from .. import types as T
    return T.RecordT([("Name", T.String), ("V1", T.Int64), ("V2", T.Int64)], tuple)
