"""Receive arena of the streamed shuffle (parallel/exchange.RecvArena): consecutive rounds land
back to back per column, so their tables concatenate as one view; a round that does not fit, or
whose column layout differs, gets fresh buffers."""
import torch

from dryad_amd.gpu.table import DeviceTable, Shape
from dryad_amd.parallel import exchange as EXC
from dryad_amd.parallel import shuffle


def _round(arena, n, base):
    slots = arena.take({"k": 8, "c": 4}, n)
    if slots is None:
        return None
    k = slots["k"].view(torch.int64)
    c = slots["c"].view(torch.int32)
    k.copy_(torch.arange(base, base + n))
    c.fill_(base)
    return DeviceTable(n, Shape("partial", ["k", "c"]), {"k": k, "c": c})


def test_rounds_concatenate_as_one_view():
    a = EXC.RecvArena(12 * 100, torch.device("cpu"))           # room for 100 rows of 12 bytes
    t1, t2 = _round(a, 40, 0), _round(a, 50, 40)
    assert t1 is not None and t2 is not None
    cat = DeviceTable.concat([t1, t2])
    assert cat.n == 90 and cat.cols["k"].data_ptr() == t1.cols["k"].data_ptr()       # a view, no copy
    assert torch.equal(cat.cols["k"], torch.arange(90))
    assert _round(a, 20, 90) is None                          # past the arena: fresh buffers
    assert a.take({"k": 8}, 1) is None                         # another column layout


def test_gather_json_single_process():
    assert shuffle.gather_json({"a": [1, 2], 3: "x"}) == [{"a": [1, 2], "3": "x"}]
