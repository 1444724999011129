"""Tiny flagship job through the public API on one GPU (used by __graft_entry__.smoke)."""
from __future__ import annotations


def run_smoke(device="cuda:0"):
    import torch
    import dryad_amd as D
    from dryad_amd.ops import terasort as TS

    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = 1
    n = 1 << 16
    q = ctx.FromStore(f"gen://terasort?records={n}&partitions=1&seed=99").OrderBy(lambda r: r[0:10])
    q.ToStore("hbm://smoke_out", delete_if_exists=True).SubmitAndWait()
    from dryad_amd.io.providers import provider_for
    rows = provider_for("hbm://smoke_out").get("hbm://smoke_out")["local"][0].rows
    acc = TS.check(rows)
    assert rows.shape[0] == n and int(acc[1]) == 0, "TeraSort smoke: output not sorted"
    # a columnar GroupBy-aggregate through the device operators
    data = [(i % 13, float(i)) for i in range(10_000)]
    got = sorted(ctx.FromEnumerable(data).GroupBy(lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1]))))
    exp = sorted((k, sum(1 for d in data if d[0] == k), float(sum(d[1] for d in data if d[0] == k))) for k in range(13))
    assert [(a, b) for a, b, _ in got] == [(a, b) for a, b, _ in exp]
    assert all(abs(x[2] - y[2]) < 1e-6 * max(1.0, abs(y[2])) for x, y in zip(got, exp))
    ex = ctx._get_executor()
    torch.cuda.synchronize()
    return ex.last_result
