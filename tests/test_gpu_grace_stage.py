"""General grace hash join stage (runtime/grace_stage.py): any Join (not only the linear-Sum
idiom of the fused join) over gen / partfile / hbm inputs, partitioned into hash buckets with
spill to pinned host DRAM past the HBM budget, the rest of the stage run per bucket; results
against the LocalDebug oracle, no host fallbacks."""
import pytest

import dryad_amd as D

pytestmark = pytest.mark.gpu

R = "gen://records64?count=200000&partitions={P}&keys=200000&seed=3&mode=dim"
S = "gen://records64?count=300000&partitions={P}&keys=200000&seed=4"


def _ctx(P=2, budget=None):
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = P
    c.GraceJoin = True
    if budget is not None:
        c.HbmBudgetBytes = budget
    return c


def _loc():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def _same(got, exp):
    """Equal record lists, reported briefly (the full diff of 1e5-record lists takes minutes)."""
    if got == exp:
        return
    bad = next(i for i, (a, b) in enumerate(zip(got, exp)) if a != b) if len(got) == len(exp) else None
    raise AssertionError(f"{len(got)} vs {len(exp)} records; first difference at {bad}: "
                         f"{got[bad] if bad is not None else got[:3]} vs {exp[bad] if bad is not None else exp[:3]}")


def _stats(c):
    r = c._get_executor().last_result
    return r, r.get("join") or {}


@pytest.mark.parametrize("budget", [None, 6 << 20])
def test_join_select_to_partfile_streams_buckets(tmp_path, budget):
    g = _ctx(budget=budget)
    uri = "partfile://" + str(tmp_path / "j.pt")
    q = lambda c: c.FromStore(R.format(P=2)).Join(c.FromStore(S.format(P=2)), lambda r: r[0], lambda s: s[0],  # noqa
                                                   lambda r, s: (r[0], r[1], s[2]))
    q(g).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    res, js = _stats(g)
    assert js.get("kind") == "grace join stage", js
    assert res["fallbacks"] == [], res["fallbacks"]
    assert js["written_bytes"] > 0
    if budget is not None:
        assert js["spilled_bytes"] > 0 and not js["in_hbm"], js
    got = sorted(g.FromStore(uri))
    exp = sorted(q(_loc()))
    _same(got, exp)
    assert len(got) == 300000


def test_join_float_sum_and_groupby_after_join():
    g = _ctx(budget=6 << 20)
    q = lambda c: c.FromStore(R.format(P=2)).Join(c.FromStore(S.format(P=2)), lambda r: r[0], lambda s: s[0],  # noqa
                                                   lambda r, s: r[1] * 0.5 + s[2] * 0.25).Sum()
    got, exp = q(g), q(_loc())
    assert abs(got - exp) <= 1e-9 * abs(exp)
    _, js = _stats(g)
    assert js.get("kind") == "grace join stage" and js["spilled_bytes"] > 0
    q2 = lambda c: c.FromStore(R.format(P=2)).Join(  # noqa
        c.FromStore(S.format(P=2)), lambda r: r[0], lambda s: s[0], lambda r, s: (r[1] % 97, s[2])).GroupBy(
        lambda t: t[0], lambda k, grp: (k, grp.Count(), grp.Sum(lambda t: t[1])))
    _same(sorted(q2(g)), sorted(q2(_loc())))
    assert _stats(g)[0]["fallbacks"] == []


def test_join_partfile_and_hbm_inputs(tmp_path):
    g = _ctx()
    ru, su = "partfile://" + str(tmp_path / "r.pt"), "partfile://" + str(tmp_path / "s.pt")
    g.FromStore(R.format(P=2)).ToStore(ru, delete_if_exists=True).SubmitAndWait()
    g.FromStore(S.format(P=2)).Select(lambda s: (s[0], s[2] * 1.5, s[3])).ToStore(su, delete_if_exists=True) \
        .SubmitAndWait()
    q = lambda c, a, b: c.FromStore(a).Join(c.FromStore(b), lambda r: r[0], lambda s: s[0],  # noqa
                                            lambda r, s: (r[0], s[1] + r[2]))
    got = sorted(q(g, ru, su))
    assert _stats(g)[1].get("kind") == "grace join stage"
    exp = sorted(q(_loc(), R.format(P=2), "x") if False else
                 _loc().FromStore(R.format(P=2)).Join(_loc().FromStore(S.format(P=2)).Select(
                     lambda s: (s[0], s[2] * 1.5, s[3])), lambda r: r[0], lambda s: s[0],
                     lambda r, s: (r[0], s[1] + r[2])))
    _same(got, exp)
    hb = "hbm://grace_side"
    g.FromStore(S.format(P=2)).Select(lambda s: (s[0], s[1])).ToStore(hb, delete_if_exists=True).SubmitAndWait()
    got = sorted(g.FromStore(R.format(P=2)).Join(g.FromStore(hb), lambda r: r[0], lambda s: s[0],
                                                  lambda r, s: (r[1], s[1])))
    assert _stats(g)[1].get("kind") == "grace join stage"
    exp = sorted(_loc().FromStore(R.format(P=2)).Join(_loc().FromStore(S.format(P=2)).Select(
        lambda s: (s[0], s[1])), lambda r: r[0], lambda s: s[0], lambda r, s: (r[1], s[1])))
    _same(got, exp)


def test_join_to_partfile_recovers_from_a_bucket_failure(tmp_path, monkeypatch):
    """A bucket that fails after earlier buckets were streamed into the output part file: the
    stage's writer is aborted (the process-wide writer ring released, the partial part removed),
    so the compiled stages that take over (the failure hit every rank) open their own writer and
    the job completes oracle-equal."""
    from dryad_amd.ops import grace as GR
    real = GR.hash_join_pairs
    calls = {"n": 0}

    def flaky(*a, **k):
        calls["n"] += 1
        if calls["n"] == 3:                  # the third bucket of the first attempt
            raise RuntimeError("injected bucket failure")
        return real(*a, **k)
    monkeypatch.setattr(GR, "hash_join_pairs", flaky)
    g = _ctx()
    uri = "partfile://" + str(tmp_path / "jf.pt")
    q = lambda c: c.FromStore(R.format(P=2)).Join(c.FromStore(S.format(P=2)), lambda r: r[0], lambda s: s[0],  # noqa
                                                   lambda r, s: (r[0], r[1], s[2]))
    q(g).ToStore(uri, delete_if_exists=True).SubmitAndWait()      # (hung in PartWriter before the fix)
    assert calls["n"] >= 3
    import os
    parts_dir = str(tmp_path / "jf.pt.parts")
    assert not [f for f in os.listdir(parts_dir) if f.endswith(".tmp")], os.listdir(parts_dir)
    _same(sorted(g.FromStore(uri)), sorted(q(_loc())))
