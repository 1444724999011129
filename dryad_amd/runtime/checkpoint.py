"""Persisted stage outputs: what lets a relaunched gang resume a job after a lost rank process.

The reference survives the loss of a vertex process because every vertex output is a file that
outlives it: a failed vertex is re-executed from its persisted inputs (DrActiveVertex::
ReactToFailedVertex, GraphManager/vertex/DrVertex.cpp:1042-1171; DrGraph::ReportFailure,
DrGraph.cpp:392-456), and a partition becomes visible only through commit-by-rename
(DrPartitionFile.cpp:496-600).  Here channels live in HBM, inside the rank processes; when one of
them dies the launcher (csrc/launcher/dryad_launch.cpp) stops the gang and starts a fresh one,
and the job's stages whose outputs were persisted here are not run again.

Layout: ``<root>/<job key>/s<stage>/p<partition>.{pt,json,pkl}`` plus a ``.done`` marker written
by rename after the data files, so a rank that died mid-write leaves no partial checkpoint.  The
job key is the job's sequence number in the process plus a digest of its plan: a relaunched
script submits the same jobs in the same order.  Device tables are tensor files (loaded with
``torch.load(weights_only=True)``) with a JSON layout; host record lists are pickles this
framework wrote itself.
"""
from __future__ import annotations

import hashlib
import json
import os
import pickle
import uuid

import torch

from ..gpu.table import DeviceTable, Ported, PortTables
from ..tools.replay import _shape_from, _shape_json


def job_key(seq: int, plan) -> str:
    """Stable across processes and relaunches: the job's order in the script and its plan's
    structure (stage names, partition counts, edges, operator names; not lambda reprs or the
    generated names of temporary outputs, which differ between processes)."""
    shape = [(s.name, s.partitions, [(i.src, i.kind) for i in s.inputs], [o["op"] for o in s.ops])
             for s in plan.stages]
    d = hashlib.blake2b(repr(shape).encode(), digest_size=8).hexdigest()
    return f"job{seq:04d}-{d}"


def _table_tensors(t: DeviceTable) -> tuple[dict, dict]:
    tensors = {"col:" + c: v[: t.n].detach().cpu() for c, v in t.cols.items()}
    if t.rows is not None:
        tensors["rows"] = t.rows[: t.n].detach().cpu()
    if t.heap is not None:
        tensors["heap"] = t.heap.detach().cpu()
    for f_, h in t.strs.items():
        tensors["str:" + f_] = h.detach().cpu()
    return tensors, dict(n=t.n, shape=_shape_json(t.shape), cols=list(t.cols))


def _table_from(tensors: dict, meta: dict, device, prefix: str = "") -> DeviceTable:
    g = lambda k: tensors.get(prefix + k)  # noqa: E731
    cols = {c: g("col:" + c).to(device) for c in meta["cols"]}
    strs = {k[len(prefix) + 4:]: v.to(device) for k, v in tensors.items() if k.startswith(prefix + "str:")}
    rows, heap = g("rows"), g("heap")
    return DeviceTable(meta["n"], _shape_from(meta["shape"]), cols,
                       rows=rows.to(device) if rows is not None else None,
                       heap=heap.to(device) if heap is not None else None, strs=strs)


class StageCheckpoint:
    def __init__(self, root: str, key: str):
        self.dir = os.path.join(root, key)

    def _base(self, sid: int, p: int) -> str:
        return os.path.join(self.dir, f"s{sid}", f"p{p}")

    def drop(self, sid: int, p: int) -> None:
        base = self._base(sid, p)
        for ext in (".done", ".json", ".pt", ".pkl"):          # the marker first: never half a checkpoint
            try:
                os.remove(base + ext)
            except OSError:
                pass

    def has(self, sid: int, p: int) -> bool:
        return os.path.exists(self._base(sid, p) + ".done")

    @staticmethod
    def persistable(value) -> bool:
        if value is None or isinstance(value, DeviceTable):
            return True
        if isinstance(value, Ported):
            return isinstance(value.table, DeviceTable)
        if isinstance(value, PortTables):
            return all(x is None or isinstance(x, (DeviceTable, list)) for x in value.tables)
        return isinstance(value, list)

    def save(self, sid: int, p: int, value) -> bool:
        """Persist one vertex output (False: a kind this store does not hold; the stage then
        simply runs again after a relaunch)."""
        if not self.persistable(value):
            return False
        base = self._base(sid, p)
        os.makedirs(os.path.dirname(base), exist_ok=True)
        tag = uuid.uuid4().hex[:8]
        meta: dict = {}
        tensors: dict = {}
        obj = None
        if value is None:
            meta["kind"] = "none"
        elif isinstance(value, DeviceTable):
            tensors, meta["table"] = _table_tensors(value)
            meta["kind"] = "table"
        elif isinstance(value, Ported):
            tensors, meta["table"] = _table_tensors(value.table)
            meta.update(kind="ported", offsets=list(value.offsets), order=value.order)
        elif isinstance(value, PortTables):
            meta.update(kind="port_tables", ports=[])
            objs = []
            for k, x in enumerate(value.tables):
                if isinstance(x, DeviceTable):
                    tk, mk = _table_tensors(x)
                    tensors.update({f"{k}/{n}": v for n, v in tk.items()})
                    meta["ports"].append(dict(kind="table", table=mk))
                else:
                    meta["ports"].append(dict(kind="objects", index=len(objs)))
                    objs.append(x)
            obj = objs
        else:
            meta["kind"] = "objects"
            obj = value
        if tensors:
            torch.save(tensors, f"{base}.pt.{tag}")
            os.replace(f"{base}.pt.{tag}", base + ".pt")
        if obj is not None:
            with open(f"{base}.pkl.{tag}", "wb") as f:
                pickle.dump(obj, f)
            os.replace(f"{base}.pkl.{tag}", base + ".pkl")
        with open(f"{base}.json.{tag}", "w") as f:
            json.dump(meta, f)
        os.replace(f"{base}.json.{tag}", base + ".json")
        with open(f"{base}.done.{tag}", "w") as f:
            f.write("1")
        os.replace(f"{base}.done.{tag}", base + ".done")            # commit by rename
        return True

    def load(self, sid: int, p: int, device):
        base = self._base(sid, p)
        with open(base + ".json") as f:
            meta = json.load(f)
        kind = meta["kind"]
        tensors = torch.load(base + ".pt", weights_only=True) if os.path.exists(base + ".pt") else {}
        obj = None
        if os.path.exists(base + ".pkl"):
            with open(base + ".pkl", "rb") as f:           # written by this framework (save above)
                obj = pickle.load(f)
        if kind == "none":
            return None
        if kind == "table":
            return _table_from(tensors, meta["table"], device)
        if kind == "ported":
            return Ported(_table_from(tensors, meta["table"], device), meta["offsets"], meta["order"])
        if kind == "port_tables":
            tabs = []
            for k, pm in enumerate(meta["ports"]):
                tabs.append(_table_from(tensors, pm["table"], device, prefix=f"{k}/") if pm["kind"] == "table"
                            else obj[pm["index"]])
            return PortTables(tabs)
        return obj


def from_env(ctx):
    """The checkpoint root when stage outputs are to be persisted: the context's
    PersistStageOutputs (a directory, or True for DRYAD_CHECKPOINT_DIR), or automatically under a
    launcher that relaunches lost gangs (DRYAD_GANG_RESTARTS > 0).  None: no persistence."""
    want = ctx._props.get("PersistStageOutputs")
    if want is False:
        return None
    if isinstance(want, str):
        return want
    root = os.environ.get("DRYAD_CHECKPOINT_DIR")
    if want or (root and int(os.environ.get("DRYAD_GANG_RESTARTS", "0") or 0) > 0):
        if not root:
            from .executor import dryad_home
            root = os.path.join(dryad_home(ctx), "checkpoints")
        return root
    return None


def gang_epoch() -> int:
    """How many times the launcher has relaunched this job's gang (0: the first start)."""
    return int(os.environ.get("DRYAD_GANG_EPOCH", "0") or 0)
