"""BasicAPITests / SimpleTests scenarios: submission semantics, ToStore/FromStore round trips,
repeat submission, context immutability, multiple outputs, WordCount (config #1 of BASELINE.json)
through LocalJobSubmission-style CPU vertex-host processes."""
import os

import pytest

import dryad_amd as D
from dryad_amd.errors import DryadLinqException
from helpers import cluster_ctx, local_ctx


def test_tostore_submit_and_read_back(tmp_path):
    c = cluster_ctx()
    uri = f"partfile://{tmp_path}/t1"
    info = c.FromEnumerable(range(50)).Select(lambda x: x * 3).ToStore(uri).SubmitAndWait()
    assert info.status == D.JobStatus.Success
    assert sorted(c.FromStore(uri)) == [x * 3 for x in range(50)]
    # partfile metadata is byte-format compatible: base, count, idx,size lines
    lines = open(f"{tmp_path}/t1").read().splitlines()
    assert int(lines[1]) == 3 and all(len(l.split(",")) == 2 for l in lines[2:])


def test_tostore_existing_requires_delete(tmp_path):
    c = cluster_ctx()
    uri = f"partfile://{tmp_path}/t2"
    c.FromEnumerable([1]).ToStore(uri).SubmitAndWait()
    with pytest.raises(DryadLinqException):
        c.FromEnumerable([2]).ToStore(uri).SubmitAndWait()
    c.FromEnumerable([3]).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    assert list(c.FromStore(uri)) == [3]


def test_repeat_submission_returns_same_job(tmp_path):
    c = cluster_ctx()
    q = c.FromEnumerable(range(5)).ToStore(f"partfile://{tmp_path}/t3")
    a = q.Submit()
    b = q.Submit()
    assert a is b
    a.Wait()


def test_enumerate_twice_and_materialized_query(tmp_path):
    c = cluster_ctx()
    q = c.FromEnumerable(range(10)).Where(lambda x: x > 4)
    assert sorted(q) == sorted(q) == [5, 6, 7, 8, 9]
    st = q.ToStore(f"partfile://{tmp_path}/t4")
    st.SubmitAndWait()
    assert sorted(st) == [5, 6, 7, 8, 9]          # data-backed query reads the table


def test_context_config_is_read_only_after_use():
    c = D.DryadLinqContext(2)
    c._props["PoolKind"] = "thread"
    c.JobFriendlyName = "x"
    list(c.FromEnumerable([1, 2]))
    with pytest.raises(DryadLinqException):
        c.JobFriendlyName = "y"
    c.Dispose()


def test_multiple_queries_one_job(tmp_path):
    c = cluster_ctx()
    base = c.FromEnumerable(range(30))
    q1 = base.Where(lambda x: x % 2 == 0).ToStore(f"partfile://{tmp_path}/a")
    q2 = base.Where(lambda x: x % 2 == 1).ToStore(f"partfile://{tmp_path}/b")
    info = c.SubmitAndWait(q1, q2)
    assert len(info.JobIds) == 1
    assert sorted(c.FromStore(f"partfile://{tmp_path}/a")) == list(range(0, 30, 2))
    assert sorted(c.FromStore(f"partfile://{tmp_path}/b")) == list(range(1, 30, 2))


def test_speculative_duplication_toggle():
    c = D.DryadLinqContext(2)
    c.EnableSpeculativeDuplication = False
    c._props["PoolKind"] = "thread"
    assert sorted(c.FromEnumerable(range(5))) == list(range(5))
    c.Dispose()


def test_localdebug_equivalence_of_typed_outputs(tmp_path):
    for c in (local_ctx(), cluster_ctx()):
        uri = f"partfile://{tmp_path}/typed-{id(c)}"
        c.FromEnumerable([("a", 1.5), ("b", 2.5)]).ToStore(uri, delete_if_exists=True).SubmitAndWait()
        assert sorted(c.FromStore(uri)) == [("a", 1.5), ("b", 2.5)]


def _wordcount(ctx, lines_uri, out_uri):
    """samples/WordCount.cs.pp: SelectMany(split) -> GroupBy(w) -> Select(count)."""
    return (ctx.FromStore(lines_uri)
            .SelectMany(lambda l: l.Line.split(" "))
            .GroupBy(lambda w: w, lambda k, g: (k, g.Count()))
            .Select(lambda kv: D.LineRecord(f"{kv[0]}: {kv[1]}"))
            .ToStore(out_uri, delete_if_exists=True))


def test_wordcount_local_job_submission_processes(tmp_path):
    """BASELINE config #1: WordCount via LocalJobSubmission on CPU (real vertex-host processes)."""
    from dryad_amd.io.providers import provider_for
    text = ["the quick brown fox", "jumps over the lazy dog", "the end"] * 20
    src = f"partfile://{tmp_path}/lines"
    provider_for(src).write_table(src, [[D.LineRecord(t) for t in text[:30]], [D.LineRecord(t) for t in text[30:]]],
                                  D.types.LineRecordT)
    c = D.DryadLinqContext(3)        # process pool (VertexHost programs)
    out = f"partfile://{tmp_path}/wc"
    info = _wordcount(c, src, out).SubmitAndWait()
    wc_dir = c._get_executor().last_job_dir
    got = sorted(l.Line for l in c.FromStore(out, D.types.LineRecordT))
    from collections import Counter
    exp = sorted(f"{w}: {n}" for w, n in Counter(w for t in text for w in t.split(" ")).items())
    assert got == exp
    # the job left its Calypso-style event log and statistics
    ex = c._get_executor()
    assert os.path.exists(os.path.join(ex.last_job_dir, "log", "events.jsonl"))
    assert os.path.exists(os.path.join(ex.last_job_dir, "statistics.json"))
    assert any(e.get("ev") == "job_stop" for e in info.events)
    # ... and the reference-format query plan (DryadLinqQueryGen.cs:837-971)
    import xml.etree.ElementTree as ET
    root = ET.parse(os.path.join(wc_dir, "QueryPlan.xml")).getroot()
    assert root.tag == "Query" and root.find("DryadLinqVersion") is not None
    verts = root.findall("./QueryPlan/Vertex")
    assert len(verts) >= 2
    ids = {v.findtext("UniqueId") for v in verts}
    for v in verts:
        assert {e.tag for e in v} >= {"UniqueId", "Type", "Name", "Explain", "Partitions", "ChannelType",
                                      "ConnectionOperator", "DynamicManager", "Entry", "Children"}
        for ch in v.findall("./Children/Child"):
            assert ch.findtext("UniqueId") in ids and ch.findtext("AffinityConstraint") == "UseDefault"
    assert any(v.findtext("ConnectionOperator") == "CrossProduct" for v in verts)    # the word shuffle
    c.Dispose()
