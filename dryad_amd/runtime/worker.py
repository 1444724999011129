"""Vertex host: executes vertex commands for the CPU executor.

Reference: DryadVertex/VertexHost (VertexHost.exe: vertexHost.cpp:252-364 -> DryadVertexMain ->
DVertexPnController::ActOnCommand Start/Terminate, dvertexpncontrol.cpp:737-961) and the
ProcessService that launches it.  A worker process is long-lived (one per slot); the job manager
sends it ``VertexCommand`` dicts over a pipe, the worker reads its input channels, runs the vertex
program and writes its output channels, then replies with a status dict.  Failures are reported,
never raised: an exception while *reading* an input channel is blamed on that channel's edge
(``bad_edge``) so the job manager re-executes the producer (DrGraph::ReportFailure).

Fault injection (the reference's FakeVertexFailure flags were never wired up): a
command may carry ``faults`` = list of {stage, partition, version, kind} with kind in
``fail`` (raise), ``read_error`` (fail reading input 0), ``slow:<seconds>``, ``crash`` (exit the
worker process).
"""
from __future__ import annotations

import gzip
import os
import pickle
import sys
import time
import traceback

from . import vertex_ops as V

_PLAN_CACHE: dict = {}


class ChannelReadError(Exception):
    def __init__(self, edge, msg):
        super().__init__(msg)
        self.edge = edge


def load_plan(job_dir: str):
    p = _PLAN_CACHE.get(job_dir)
    if p is None:
        import cloudpickle  # noqa: F401  (registers reducers used by the pickle)
        with open(os.path.join(job_dir, "plan.pkl"), "rb") as f:
            p = pickle.load(f)
        _PLAN_CACHE.clear()
        _PLAN_CACHE[job_dir] = p
    return p


def read_channel(path: str, edge: int):
    try:
        with open(path, "rb") as f:
            data = f.read()
        if data[:2] == b"\x1f\x8b":
            data = gzip.decompress(data)
        return pickle.loads(data), len(data)
    except Exception as e:  # noqa: BLE001
        raise ChannelReadError(edge, f"cannot read channel {path}: {e}")


def write_channel(path: str, records, compress: bool = False) -> int:
    data = pickle.dumps(records, protocol=pickle.HIGHEST_PROTOCOL)
    if compress:
        data = gzip.compress(data, compresslevel=1)
    tmp = path + ".partial"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)
    return len(data)


def _fault(cmd, stage):
    for f in cmd.get("faults") or ():
        if f.get("stage") not in (None, stage.id, stage.name):
            continue
        if f.get("partition") not in (None, cmd["partition"]):
            continue
        if f.get("version") not in (None, cmd["version"]):
            continue
        return f.get("kind", "fail")
    return None


def _merge_inputs(stage_input, streams):
    if stage_input.merge_sort:
        ms = stage_input.merge_sort
        return list(V.E.MergeSort(streams, ms["key"], ms.get("comparer"), ms.get("descending", False)))
    if len(streams) == 1:
        return streams[0]
    return [x for s in streams for x in s]


def write_output_part(stage, records, path: str, compress=False, output_gzip=False):
    """Write an output partition in the DryadLinqBinary record format (typed) or pickle."""
    from .. import types as T
    from ..io import binary as B
    dtype = stage.output.get("dtype") or stage.dtype
    if dtype is None or dtype == T.Pickle:
        dtype = T.infer_common_type(records[:1000]) if records else None
    uri = stage.output["uri"]
    if not records and (dtype is None or dtype == T.Pickle) and not stage.output.get("temp"):
        # an empty partition of an untyped output: a 0-byte part reads back as [] in every format,
        # so it must not force the whole table to the pickle format
        with open(path, "wb"):
            pass
        return 0, None, None
    from ..io.providers import parse_uri
    if stage.output.get("temp") or parse_uri(uri)[0] not in ("partfile", "file") or dtype is None \
            or dtype == T.Pickle:
        # non-partfile stores are committed by their provider from the channel records
        n = write_channel(path, records, compress)
        return n, (dtype.name if dtype is not None else None), "pickle"
    ser = stage.output.get("serializer")
    if ser is not None:
        with open(path, "wb") as f:
            ser(records, f)
        return os.path.getsize(path), dtype.name, "custom"
    if output_gzip:
        # whole-stream gzip of the record stream (CompressionScheme.Gzip,
        # DryadLinqBlockStream.cs:198-225); readers detect the gzip magic
        data = gzip.compress(B.encode_records(dtype, records), compresslevel=6)
        with open(path, "wb") as f:
            f.write(data)
        return len(data), dtype.name, "binary"
    n = B.write_records(path, dtype, records)
    return n, dtype.name, "binary"


def execute_vertex(cmd: dict, plan=None) -> dict:
    t0 = time.time()
    res = dict(vertex=cmd["vertex"], version=cmd["version"], ok=False, error=None, bad_edge=-1, bytes_read=0,
               bytes_written=0, records_out=0, dtype=None, fmt=None, pid=os.getpid())
    try:
        plan = plan or load_plan(cmd["job"])
        stage = plan.stages[cmd["stage"]]
        fault = _fault(cmd, stage)
        if fault == "crash":
            os._exit(17)
        if fault and fault.startswith("slow"):
            time.sleep(float(fault.split(":")[1]) if ":" in fault else 1.0)
        inputs = []
        for si, chans in zip(stage.inputs, cmd["inputs"]):
            streams = []
            for path, edge in chans:
                if fault == "read_error" and not inputs and not streams:
                    raise ChannelReadError(edge, f"injected read error on {path}")
                recs, nb = read_channel(path, edge)
                res["bytes_read"] += nb
                streams.append(recs)
            inputs.append(_merge_inputs(si, streams) if streams else [])
        if fault == "fail":
            raise RuntimeError(f"injected vertex failure {stage.name}[{cmd['partition']}] v{cmd['version']}")
        vctx = V.VertexContext(cmd["partition"], stage.partitions, cmd["vertex"], cmd["version"], stage)
        out = V.run_program(stage.ops, inputs, vctx)
        ports = out if stage.out_ports > 1 else [out]
        compress = bool(cmd.get("compress"))
        if stage.is_output:
            recs = ports[0]
            nb, dt, fmt = write_output_part(stage, recs, cmd["output_part"], compress, bool(cmd.get("output_gzip")))
            res.update(bytes_written=nb, dtype=dt, fmt=fmt, records_out=len(recs))
        else:
            for k, path in enumerate(cmd["outputs"]):
                recs = ports[k] if k < len(ports) else []
                res["bytes_written"] += write_channel(path, recs, compress)
                res["records_out"] += len(recs)
        res["ok"] = True
    except ChannelReadError as e:
        res["error"] = str(e)
        res["bad_edge"] = e.edge
    except BaseException as e:  # noqa: BLE001
        res["error"] = f"{type(e).__name__}: {e}\n{traceback.format_exc(limit=8)}"
        res["exc"] = _safe_exc(e)
    res["elapsed"] = time.time() - t0
    return res


def _safe_exc(e):
    try:
        pickle.dumps(e)
        return e
    except Exception:
        return None


def worker_main(conn, slot: int):
    """Worker process loop (one per slot)."""
    os.environ["DRYAD_WORKER_SLOT"] = str(slot)
    while True:
        try:
            cmd = conn.recv()
        except (EOFError, OSError):
            return
        if cmd is None:
            return
        if isinstance(cmd, tuple):      # handshake / control messages
            continue
        res = execute_vertex(cmd)
        try:
            conn.send(res)
        except (BrokenPipeError, OSError):
            return


if __name__ == "__main__":  # pragma: no cover - manual replay of one vertex command
    import json
    cmd = json.load(open(sys.argv[1]))
    print(execute_vertex(cmd))
