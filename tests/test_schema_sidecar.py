"""The partfile ``.dryadtype`` sidecar is declarative JSON (no code runs when a foreign table's
schema is read), opaque pickled tables from other processes are refused, and error codes of
common API misuse are the reference's."""
import dataclasses
import json
import os

import pytest

import dryad_amd as D
from dryad_amd import types as T
from dryad_amd.errors import DryadLinqException, ErrorCode
from dryad_amd.runtime import jobmanager as JM


@dataclasses.dataclass
class Person:
    name: str
    age: int
    score: float


@pytest.mark.parametrize("dt", [T.Int32, T.String, T.LineRecordT, T.Nullable(T.Int64), T.ArrayT(T.Byte),
                                T.Vector(T.Float32, 8), T.record_type(Person),
                                T.RecordT([("Item1", T.Int64), ("Item2", T.String)], tuple), T.Pickle])
def test_dtype_json_round_trip(dt):
    assert T.dtype_from_json(json.loads(json.dumps(T.dtype_to_json(dt)))) == dt


def test_record_class_resolved_only_from_loaded_modules():
    o = T.dtype_to_json(T.record_type(Person))
    assert T.dtype_from_json(o).pytype is Person
    o["pytype"] = "some_module_that_is_not_imported:Evil"
    assert T.dtype_from_json(o).pytype is tuple


def test_sidecar_is_json_and_legacy_pickle_ignored(tmp_path):
    meta = str(tmp_path / "t.pt")
    JM.write_schema(meta, T.record_type(Person), "binary")
    with open(JM.schema_path(meta)) as f:
        assert json.load(f)["format"] == "binary"
    assert JM.read_schema(meta)["dtype"] == T.record_type(Person)
    with open(JM.schema_path(meta), "wb") as f:
        f.write(b"\x80\x04\x95 not json")
    assert JM.read_schema(meta) is None


def test_partfile_round_trip_through_api(tmp_path):
    ctx = D.DryadLinqContext(1)
    ctx.LocalDebug = True
    uri = "partfile://" + str(tmp_path / "people.pt")
    people = [Person("a" * (i % 5), i, i / 2) for i in range(50)]
    ctx.FromEnumerable(people).ToStore(uri).SubmitAndWait()
    assert list(ctx.FromStore(uri)) == people


def test_foreign_pickled_table_refused(tmp_path, monkeypatch):
    meta = str(tmp_path / "opaque.pt")
    from dryad_amd.io import partfile as PF
    import pickle
    base = PF.default_base(meta)
    os.makedirs(os.path.dirname(base), exist_ok=True)
    tmp = PF.tmp_part_path(base, 0, 0, 0, 0)
    with open(tmp, "wb") as f:
        f.write(pickle.dumps([object.__new__(object)]))
    PF.commit_parts(meta, base, [tmp])
    with open(JM.schema_path(meta), "w") as f:
        json.dump({"dtype": {"t": "Pickle"}, "format": "pickle"}, f)
    ctx = D.DryadLinqContext(1)
    ctx.LocalDebug = True
    with pytest.raises(DryadLinqException) as ei:
        list(ctx.FromStore("partfile://" + meta))
    assert ei.value.error_code == ErrorCode.FailedToDeserialize
    monkeypatch.setenv("DRYAD_TRUST_PICKLED_TABLES", "1")
    assert len(list(ctx.FromStore("partfile://" + meta))) == 1


def test_reference_error_codes():
    c1, c2 = D.DryadLinqContext(1), D.DryadLinqContext(platform="gpu")
    c1.LocalDebug = True
    with pytest.raises(DryadLinqException) as ei:
        c1.FromEnumerable([1]).Concat(c2.FromEnumerable([2]))
    assert ei.value.error_code == ErrorCode.MustStartFromContext
    with pytest.raises(DryadLinqException) as ei:
        c1.FromEnumerable([1, 2]).SlidingWindow(lambda w: w, 1)
    assert ei.value.error_code == ErrorCode.Unspecified == 0     # reference: message-only ctor
    with pytest.raises(DryadLinqException) as ei:
        c1.FromEnumerable([]).First()
    assert ei.value.error_code in (ErrorCode.FirstNoElementsFirst, ErrorCode.AggregateNoElements)
    with pytest.raises(DryadLinqException) as ei:
        c1.FromEnumerable([1, 2]).Single()
    assert ei.value.error_code == ErrorCode.SingleMoreThanOneElement


def test_gpu_runner_fallback_guard_without_gpu():
    """GpuJobRunner._fallback (the host-fallback size guard) on a stub runner."""
    import torch
    from types import SimpleNamespace
    from dryad_amd.gpu.table import DeviceTable, Shape
    from dryad_amd.runtime.gpu_executor import GpuJobRunner
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.HostFallbackMaxBytes = 1 << 20
    t = DeviceTable.from_columns({"v": torch.zeros(1 << 20, dtype=torch.int64)}, Shape("scalar", ["v"]))
    r = SimpleNamespace(fallbacks=[], gpu_ok=True, ctx=ctx)
    st = SimpleNamespace(name="s0")
    with pytest.raises(DryadLinqException) as ei:
        GpuJobRunner._fallback(r, st, "aggregate_seq", "not traceable", [t])
    assert ei.value.error_code == ErrorCode.OperatorNotSupported
    ctx2 = D.DryadLinqContext(platform="gpu")
    ctx2.AllowHostFallback = True
    r2 = SimpleNamespace(fallbacks=[], gpu_ok=True, ctx=ctx2)
    GpuJobRunner._fallback(r2, st, "aggregate_seq", "not traceable", [t])
    assert r2.fallbacks == [("s0", "aggregate_seq", "not traceable")]


def test_index_sidecar_validation(tmp_path):
    """read_index refuses offsets a block-parallel decoder must not trust: not starting at 0,
    decreasing, or past the part's end."""
    import numpy as np
    from dryad_amd.io import partfile as PF
    part = str(tmp_path / "p.00000000")
    with open(part, "wb") as f:
        f.write(b"\0" * 1000)
    good = np.array([0, 100, 250, 900], dtype=np.int64)
    PF.write_index(part, 16, 1000, good, 4)
    assert PF.read_index(part) is not None
    for bad in ([5, 100, 250, 900], [0, 300, 250, 900], [0, 100, 250, 1001]):
        PF.write_index(part, 16, 1000, np.array(bad, dtype=np.int64), 4)
        assert PF.read_index(part) is None, bad
