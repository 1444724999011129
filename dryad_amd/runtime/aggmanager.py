"""Dynamic aggregation grouping (reference: GraphManager/stagemanager/DrDynamicAggregateManager.cpp
``ConsiderSending`` :470-489, ``SendMinimum`` :502-560, the singleton rule :1424-1455; thresholds
from DryadLinqGraphManager/GraphBuilder.cs:565-570 and the ``at/aggregatethreshold`` option of
DryadLinqApplication.cs:143-175, default 1 GB).

The partial-aggregate outputs of an aggregation tree level are grouped by their ACTUAL sizes once
they exist, instead of by a fixed fan-in: sources are taken in order and added to the open group
until one more would exceed ``max_inputs`` members or ``threshold`` bytes, which closes the group;
a source of at least ``threshold / 2`` bytes (the reference's maxDataToConsiderGrouping) is never
grouped, it forms a group of its own.  Groups are contiguous runs of sources in partition order,
assigned to the combine vertices in order, so the fold order of the static tree is kept.  Small partials (the common case: a Count or Sum partial is a
few bytes) thus meet in few wide combine vertices, large ones stay apart and are combined in
parallel."""
from __future__ import annotations

import re

DEFAULT_THRESHOLD = 1 << 30

_SUFFIX = {"": 1, "b": 1, "k": 1 << 10, "kb": 1 << 10, "m": 1 << 20, "mb": 1 << 20, "g": 1 << 30, "gb": 1 << 30,
           "t": 1 << 40, "tb": 1 << 40}


def parse_size(v) -> int:
    """Bytes from an int or a string with an optional size suffix ("512MB", "1g", "4096")."""
    # the reference rejects an unparsable or non-positive value (DryadLinqApplication.cs:297-313);
    # like the operator overloads' ArgumentOutOfRange this is a ValueError, not a Dryad fault code
    if isinstance(v, bool):
        raise ValueError(f"aggregate threshold: not a size: {v!r}")
    if isinstance(v, (int, float)):
        n = int(v)
    else:
        m = re.fullmatch(r"\s*(\d+(?:\.\d+)?)\s*([a-zA-Z]*)\s*", str(v))
        if m is None or m.group(2).lower() not in _SUFFIX:
            raise ValueError(f"aggregate threshold: not a size: {v!r}")
        n = int(float(m.group(1)) * _SUFFIX[m.group(2).lower()])
    if n <= 0:
        raise ValueError(f"aggregate threshold must be positive: {v!r}")
    return n


def dynamic_groups(sizes: list[int], max_inputs: int, threshold: int) -> list[list[int]]:
    """Indices of ``sizes`` grouped greedily in order (see the module docstring)."""
    max_inputs = max(1, int(max_inputs))
    single = threshold // 2
    groups: list[list[int]] = []
    cur: list[int] = []
    cur_bytes = 0
    for i, b in enumerate(sizes):
        if b >= single:                   # never grouped; groups stay contiguous runs of sources,
            if cur:                       # so an associative but order-sensitive fold keeps its order
                groups.append(cur)
                cur, cur_bytes = [], 0
            groups.append([i])
            continue
        if cur and (len(cur) == max_inputs or cur_bytes + b > threshold):
            groups.append(cur)
            cur, cur_bytes = [], 0
        cur.append(i)
        cur_bytes += b
    if cur:
        groups.append(cur)
    return groups


def assign_groups(sizes: list[int], slots: int, max_inputs: int, threshold: int) -> list[list[int]]:
    """``slots`` lists of source indices (combine vertex j reads list j; trailing lists may be
    empty).  When the size rule yields more groups than there are combine vertices, the sources
    are split into ``slots`` contiguous groups of near-equal bytes instead."""
    groups = dynamic_groups(sizes, max_inputs, threshold)
    if len(groups) > slots:
        total = sum(sizes)
        groups, cur, acc = [], [], 0
        for i, b in enumerate(sizes):
            cur.append(i)
            acc += b
            need_after = slots - len(groups) - 1          # groups still to open after this one
            if need_after > 0 and (len(sizes) - i - 1 == need_after or acc * slots >= total * (len(groups) + 1)):
                groups.append(cur)
                cur = []
        if cur:
            groups.append(cur)
    return groups + [[] for _ in range(slots - len(groups))]
