"""runtime/stream_agg.DenseState folding a stream whose chunks mix raw partials (one row per
record, counts as int8 ones) and folded partials (int64 counts): every chunk's count columns are
read by that chunk's own dtype.  CPU tensors take the torch fold path."""
import torch

from dryad_amd.gpu.table import DeviceTable, PartialMeta, Shape
from dryad_amd.runtime.stream_agg import DenseState


class _Agg:
    def __init__(self, kind):
        self.kind = kind


class _Decomp:
    aggs = [_Agg("count"), _Agg("sum"), _Agg("min"), _Agg("avg")]


def _raw(keys, vals):
    n = len(keys)
    ones = torch.ones(n, dtype=torch.int8)
    cols = {"k0": torch.tensor(keys, dtype=torch.int64), "a0": ones,
            "a1": torch.tensor(vals, dtype=torch.int64), "a2": torch.tensor(vals, dtype=torch.int64),
            "a3": torch.tensor(vals, dtype=torch.float64), "c3": ones}
    return DeviceTable.from_columns(cols, Shape("partial", list(cols), PartialMeta(1, ("count", "sum", "min", "avg"))))


def _folded(keys, vals):
    """The folded partial of (keys, vals): one row per distinct key, int64 counts."""
    g = {}
    for k, v in zip(keys, vals):
        c, s, m = g.get(k, (0, 0, None))
        g[k] = (c + 1, s + v, v if m is None else min(m, v))
    ks = sorted(g)
    cnt = torch.tensor([g[k][0] for k in ks], dtype=torch.int64)
    cols = {"k0": torch.tensor(ks, dtype=torch.int64), "a0": cnt,
            "a1": torch.tensor([g[k][1] for k in ks], dtype=torch.int64),
            "a2": torch.tensor([g[k][2] for k in ks], dtype=torch.int64),
            "a3": torch.tensor([float(g[k][1]) for k in ks], dtype=torch.float64), "c3": cnt.clone()}
    return DeviceTable.from_columns(cols, Shape("partial", list(cols), PartialMeta(1, ("count", "sum", "min", "avg"))))


def test_raw_first_chunk_then_folded_chunks():
    torch.manual_seed(0)
    chunks, allk, allv = [], [], []
    # first chunk: distinct keys (the partial step ships raw rows); later chunks repeat keys heavily
    k0 = list(range(100, 300))
    v0 = [int(x) for x in torch.randint(-50, 50, (len(k0),))]
    chunks.append(_raw(k0, v0))
    allk += k0
    allv += v0
    for _ in range(3):
        ks = [int(x) for x in torch.randint(100, 140, (500,))]
        vs = [int(x) for x in torch.randint(-50, 50, (500,))]
        chunks.append(_folded(ks, vs))
        allk += ks
        allv += vs
    chunks.append(_raw(k0[:50], v0[:50]))      # raw again after folded ones
    allk += k0[:50]
    allv += v0[:50]

    st = DenseState(_Decomp(), budget=1 << 20)
    for c in chunks:
        assert st.add(c)
    out = st.to_partial()
    got = {int(k): (int(c), int(s), int(m), float(a), int(ac))
           for k, c, s, m, a, ac in zip(out.cols["k0"], out.cols["a0"], out.cols["a1"], out.cols["a2"],
                                        out.cols["a3"], out.cols["c3"])}
    exp = {}
    for k, v in zip(allk, allv):
        c, s, m = exp.get(k, (0, 0, None))
        exp[k] = (c + 1, s + v, v if m is None else min(m, v))
    assert set(got) == set(exp)
    for k, (c, s, m) in exp.items():
        gc, gs, gm, ga, gac = got[k]
        assert (gc, gs, gm, gac) == (c, s, m, c), (k, got[k], exp[k])
        assert abs(ga - s) < 1e-9
