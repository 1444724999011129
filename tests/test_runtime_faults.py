"""Job-manager state machine (native) and fault tolerance end to end: vertex re-execution,
upstream invalidation on channel read errors, abort after 6 failures, vertex-host crashes,
speculative duplication of stragglers."""
import os

import pytest

import dryad_amd as D
from dryad_amd.errors import DryadLinqJobException
from dryad_amd.native import runtime


def _chain():
    R = runtime()
    g = R.JobGraph()
    a = g.add_stage("a", 2)
    b = g.add_stage("b", 1)
    v0, v1 = g.add_vertex(a, 0), g.add_vertex(a, 1)
    w = g.add_vertex(b, 0)
    g.add_edge(v0, 0, w, 0)
    g.add_edge(v1, 0, w, 0)
    return g, (v0, v1, w)


def run_all(g, t=0.0):
    its = g.take_ready(100, t)
    for it in its:
        g.on_running(it.vertex, it.version, 0, t)
    return its


def test_jobgraph_ready_and_completion():
    g, (v0, v1, w) = _chain()
    g.start(0.0)
    its = run_all(g)
    assert {i.vertex for i in its} == {v0, v1}
    g.on_completed(v0, 0, 1.0)
    assert g.take_ready(10, 1.0) == []
    g.on_completed(v1, 0, 1.0)
    its = run_all(g, 2.0)
    assert [i.vertex for i in its] == [w]
    acc, _ = g.on_completed(w, 0, 3.0)
    assert acc and g.done()


def test_jobgraph_failure_retries_then_aborts():
    R = runtime()
    p = R.Params()
    p.max_failures = 3
    g = R.JobGraph(p)
    s = g.add_stage("s", 1)
    v = g.add_vertex(s, 0)
    g.start(0.0)
    for k in range(3):
        its = run_all(g, float(k))
        assert its and its[0].version == k
        out = g.on_failed(v, k, float(k), -1, "boom")
    assert out.action == 2 and g.failed() and "failed 3 times" in g.failure()


def test_jobgraph_read_error_invalidates_upstream():
    g, (v0, v1, w) = _chain()
    g.start(0.0)
    run_all(g)
    g.on_completed(v0, 0, 1.0)
    g.on_completed(v1, 0, 1.0)
    run_all(g, 2.0)
    edge_from_v1 = [e for e in g.in_edges(w) if g.edge(e)[0] == v1][0]
    out = g.on_failed(w, 0, 3.0, edge_from_v1, "read error")
    assert out.action == 1 and out.invalidated_vertex == v1
    assert g.failures(w) == 0                       # not blamed on the reader
    its = run_all(g, 4.0)
    assert [(i.vertex, i.version) for i in its] == [(v1, 1)]
    g.on_completed(v1, 1, 5.0)
    its = run_all(g, 6.0)
    assert [(i.vertex, i.version) for i in its] == [(w, 1)]


def test_jobgraph_speculative_duplicate_first_wins():
    R = runtime()
    p = R.Params()
    p.default_outlier_threshold = 5.0
    p.min_outlier_threshold = 1.0
    g = R.JobGraph(p)
    s = g.add_stage("s", 4)
    vs = [g.add_vertex(s, i) for i in range(4)]
    g.start(0.0)
    run_all(g, 0.0)
    for v in vs[:3]:
        g.on_completed(v, 0, 1.0)
    assert g.outlier_threshold(s) == pytest.approx(1.0)
    dups = g.check_duplicates(10.0)
    assert len(dups) == 1 and dups[0].vertex == vs[3] and dups[0].duplicate
    its = run_all(g, 10.0)
    acc, cancel = g.on_completed(vs[3], its[0].version, 11.0)
    assert acc and cancel == [(vs[3], 0)] and g.done()
    acc2, _ = g.on_completed(vs[3], 0, 12.0)       # the slow original finishing later is discarded
    assert not acc2


def test_jobgraph_gang_restart():
    R = runtime()
    g = R.JobGraph()
    s = g.add_stage("x", 3)
    vs = [g.add_vertex(s, i) for i in range(3)]
    g.set_gang(vs)
    g.start(0.0)
    run_all(g)
    g.on_completed(vs[0], 0, 1.0)
    out = g.on_failed(vs[1], 0, 1.0, -1, "rccl error")
    assert sorted(out.cancel) == [(vs[2], 0)]
    its = run_all(g, 2.0)
    assert sorted(i.vertex for i in its) == vs        # whole gang re-runs (new versions)


def test_scheduler_locality_delay():
    R = runtime()
    s = R.Scheduler(3, 1.0)
    s.set_busy(1)
    assert s.place([1], 0.5) == -1                    # wait for the preferred worker
    assert s.place([1], 1.5) == 0                     # then take any idle one
    assert s.place([2], 0.0) == 2


# ------------------------------------------------------------------ end-to-end through vertex hosts
def _ctx(pool="process", faults=None, **props):
    c = D.DryadLinqContext(3)
    c._props["PoolKind"] = pool
    if faults:
        c._props["FaultInjection"] = faults
    c._props.update(props)
    return c


def test_vertex_failure_is_reexecuted():
    c = _ctx(faults=[dict(stage=None, partition=1, version=0, kind="fail")])
    q = c.FromEnumerable(range(100)).Select(lambda x: x + 1)
    assert sorted(q) == list(range(1, 101))
    ex = c._get_executor()
    assert '"state": "Failed"' in open(os.path.join(ex.last_job_dir, "log", "events.jsonl")).read()
    c.Dispose()


def test_vertex_host_crash_is_recovered():
    c = _ctx(faults=[dict(stage=None, partition=0, version=0, kind="crash")])
    assert sorted(c.FromEnumerable(range(30)).Where(lambda x: x % 2 == 0)) == list(range(0, 30, 2))
    c.Dispose()


def test_read_error_reexecutes_producer():
    c = _ctx(pool="thread", faults=[dict(stage="GroupBy", partition=0, version=0, kind="read_error")])
    q = c.FromEnumerable(range(60)).GroupBy(lambda x: x % 4, lambda k, g: (k, g.Count()))
    assert sorted(q) == [(0, 15), (1, 15), (2, 15), (3, 15)]
    evs = [e for e in c._get_executor().last_result and []]
    c.Dispose()


def test_job_aborts_after_max_failures():
    c = _ctx(pool="thread", faults=[dict(stage=None, partition=0, version=None, kind="fail")])
    with pytest.raises(DryadLinqJobException) as e:
        list(c.FromEnumerable(range(10)).Select(lambda x: x))
    assert "failed 6 times" in str(e.value)
    c.Dispose()


def test_user_exception_surfaces():
    c = _ctx(pool="thread")
    with pytest.raises(DryadLinqJobException) as e:
        list(c.FromEnumerable(range(10)).Select(lambda x: 1 // (x - 5)))
    assert "ZeroDivisionError" in str(e.value)
    c.Dispose()


def test_straggler_gets_duplicated():
    c = _ctx(pool="process", faults=[dict(stage=None, partition=2, version=0, kind="slow:6")],
             OutlierThresholdSeconds=0.5)
    c.PartitionCount = 3
    q = c.FromEnumerable(range(30)).Select(lambda x: x * 2)
    import time
    t = time.time()
    assert sorted(q) == [x * 2 for x in range(30)]
    assert time.time() - t < 5.5                      # the duplicate finished before the 6 s straggler
    c.Dispose()
