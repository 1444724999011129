"""Dynamic aggregation grouping (runtime/aggmanager.py; reference DrDynamicAggregateManager.cpp
ConsiderSending :470-489 / SendMinimum :502-560 / singleton rule :1424-1455, thresholds from
GraphBuilder.cs:565-570 and the GM's at/aggregatethreshold option, DryadLinqApplication.cs:143-175)."""
import json
import os

import pytest

import dryad_amd as D
from dryad_amd.runtime.aggmanager import assign_groups, dynamic_groups, parse_size


def test_parse_size_suffixes():
    assert parse_size("512MB") == 512 << 20
    assert parse_size("1g") == 1 << 30
    assert parse_size(" 2 KB ") == 2048
    assert parse_size(4096) == 4096
    for bad in ("", "12 parsecs", "-5", 0, True):
        with pytest.raises(ValueError):
            parse_size(bad)


def test_groups_close_on_fan_in_and_bytes():
    assert [len(g) for g in dynamic_groups([10] * 400, 150, 1 << 30)] == [150, 150, 100]
    # 300-byte partials under a 1000-byte threshold: three per group; a partial of >= half the
    # threshold stays alone, and groups stay contiguous runs of sources (fold order kept)
    g = dynamic_groups([300] * 10 + [600] + [100] * 5, 150, 1000)
    assert g == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9], [10], [11, 12, 13, 14, 15]]
    assert sum(g, []) == list(range(16))


def test_assign_groups_pads_and_falls_back_to_balanced_runs():
    assert assign_groups([1] * 10, 4, 150, 1000) == [list(range(10)), [], [], []]
    big = assign_groups([700] * 10, 4, 150, 1000)         # 10 singletons > 4 combine vertices
    assert len(big) == 4 and sum(big, []) == list(range(10)) and all(big)


def _job_events(c):
    ex = c._get_executor()
    with open(os.path.join(ex.last_job_dir, "log", "events.jsonl")) as f:
        return [json.loads(line) for line in f if line.strip()]


@pytest.mark.parametrize("threshold,expect_groups", [(None, [6, 6, 6, 6, 6, 6, 4]), ("40B", None)])
def test_process_executor_regroups_partials_by_size(threshold, expect_groups):
    """40 partitions, fan-in limit 6, static groups of 4 (10 combine vertices): with the default
    1 GB threshold the tiny Sum partials meet 6 per combine vertex (7 vertices used); with a
    40-byte threshold the byte rule splits them finer.  The result matches the oracle either way,
    including the order-sensitive First / Last."""
    c = D.DryadLinqContext(2)
    c._props["PoolKind"] = "process"
    c.PartitionCount = 40
    c.AggregationTreeMaxInputs = 6
    c.AggregationTreeGroup = 4
    if threshold is not None:
        c.AggregateThreshold = threshold
    data = list(range(1, 2001))
    q = c.FromEnumerable(data)
    assert q.Sum() == sum(data)
    ev = [e for e in _job_events(c) if e.get("event") == "dynamic_aggregate"]
    assert ev, "no dynamic aggregation decision recorded"
    assert ev[0]["partials"] == 40
    if expect_groups is not None:
        assert ev[0]["groups"] == expect_groups
    else:
        assert len(ev[0]["groups"]) > 7 and max(ev[0]["groups"]) < 6
    assert q.First(lambda x: x > 1500) == 1501 and q.Last(lambda x: x < 10) == 9
    c.Dispose()
