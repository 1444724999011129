"""DeviceTable host conversions that run on CPU tensors (no GPU): string-field records, and the
partial-aggregate layout converting to the host path's (key, accumulators) pairs."""
import torch

from dryad_amd.gpu.table import DeviceTable, PartialMeta, Shape, from_objects
from dryad_amd.runtime import vertex_ops as V
from dryad_amd.compiler.decomposition import decompose


def test_string_records_roundtrip_cpu():
    recs = [("alice", 1, 2.5), ("", 2, 0.0), ("bob ✓", 3, -1.0)]
    t = from_objects(recs, None, torch.device("cpu"))
    assert set(t.strs) == {"Item1"}
    assert t.to_objects() == recs
    cat = DeviceTable.concat([t, t.take(torch.tensor([2, 0]))])
    assert cat.to_objects() == recs + [recs[2], recs[0]]


def test_partial_table_matches_host_partial_format():
    rows = [("k%d" % (i % 3), i, float(i)) for i in range(30)]
    res = lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Average(lambda r: r[2]),  # noqa: E731
                        g.Any(lambda r: r[1] > 25))
    d = decompose(res, None)
    host = V.op_group_partial(dict(key=lambda r: r[0], decomp=d), [rows], None)
    host = sorted(host)
    # the same partials in the device layout (k0 string, then accumulator columns)
    keys = [k for k, _ in host]
    enc = [k.encode() for k in keys]
    ln = torch.tensor([len(b) for b in enc])
    off = torch.tensor([0, len(enc[0]), len(enc[0]) + len(enc[1])])
    cols = {"k0": off, "k0#len": ln,
            "a0": torch.tensor([a[0] for _, a in host]),
            "a1": torch.tensor([a[1] for _, a in host]),
            "a2": torch.tensor([a[2][0] for _, a in host], dtype=torch.float64),
            "c2": torch.tensor([a[2][1] for _, a in host]),
            "a3": torch.tensor([int(a[3]) for _, a in host])}
    meta = PartialMeta(1, tuple(a.kind for a in d.aggs), "single")
    t = DeviceTable(3, Shape("partial", [f for f in cols if not f.endswith("#len")], meta), cols,
                    strs={"k0": torch.frombuffer(bytearray(b"".join(enc)), dtype=torch.uint8)})
    assert t.to_objects() == host
    # and the host final consumes them
    fin = V.op_group_final(dict(decomp=d), [t.to_objects()], None)
    assert sorted(fin) == sorted(V.op_group_final(dict(decomp=d), [host], None))
