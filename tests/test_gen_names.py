"""gen://names: the string-keyed generator, natural and fixed-length (``namelen``) names."""
import pytest
import torch

import dryad_amd as D
from dryad_amd.models import names as NM


def _loc():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def test_namelen_pads_names_to_a_fixed_length():
    base = list(_loc().FromStore("gen://names?count=500&partitions=1&keys=400&seed=2"))
    wide = list(_loc().FromStore("gen://names?count=500&partitions=1&keys=400&seed=2&namelen=64"))
    assert [r[1:] for r in base] == [r[1:] for r in wide]
    for a, b in zip(base, wide):
        assert len(b[0]) == 64 and b[0][0] == "u" and int(b[0][1:]) == int(a[0][1:])


def test_device_render_matches_host_names():
    keys = torch.tensor([0, 7, 123456789, 2 ** 62], dtype=torch.int64)
    for L in (0, 32):
        heap, off, ln = NM.render(keys, L)
        got = [bytes(heap[int(o): int(o) + int(n)].tolist()).decode() for o, n in zip(off, ln)]
        exp = ["u" + (str(k).rjust(L - 1, "0") if L else str(k)) for k in keys.tolist()]
        assert got == exp


def test_namelen_must_exceed_natural_names():
    with pytest.raises(ValueError):
        NM.namelen({"namelen": "12"})
