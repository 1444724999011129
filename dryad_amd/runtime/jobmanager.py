"""Job manager driver: runs a compiled Plan on a pool of vertex hosts through the native
``JobGraph`` state machine.

Reference control plane: GraphBuilder (DryadLinqGraphManager/GraphBuilder.cs:320-504:
one vertex set per stage, ConnectPointwise / ConnectCrossProduct), DrGraphExecutor Run/Join, vertex
start commands with channel URIs (DrVertex.cpp:356-429), completion / failure reactions, output
commit by rename (DrPartitionFile.cpp:436-600) and the Calypso event log.  The state machine
itself (versions, failure policy, duplicates, gangs) is native C++ (csrc/runtime/jobgraph.cpp).
"""
from __future__ import annotations

import json
import os
import shutil
import threading
import time

from .. import types as T
from ..errors import DryadLinqException, DryadLinqJobException, ErrorCode
from ..io import partfile as PF
from ..io.providers import parse_uri, provider_for
from ..native import runtime as native_runtime
from ..utils.log import get_logger

log = get_logger("jobmanager")


class JobRunner:
    """Builds the vertex graph of one plan and drives it to completion."""

    DUPLICATE_CHECK_MS = 500      # period of the straggler check (a pump timer, not a poll)

    def __init__(self, ctx, plan, pool, job_dir: str, handle=None, faults=None):
        self.ctx = ctx
        self.plan = plan
        self.pool = pool
        self.job_dir = job_dir
        self.handle = handle
        self.faults = faults or []
        R = native_runtime()
        p = R.Params()
        p.max_failures = int(getattr(ctx, "MaxVertexFailures", 6) or 6)
        p.speculative = bool(ctx.EnableSpeculativeDuplication)
        thr = getattr(ctx, "_props", {}).get("OutlierThresholdSeconds")
        if thr is not None:
            p.default_outlier_threshold = float(thr)
            p.min_outlier_threshold = min(p.min_outlier_threshold, float(thr))
        self.g = R.JobGraph(p)
        self.out_bytes: dict = {}     # vid -> bytes written by its accepted version
        self.dyn_groups: dict = {}    # (stage id, input index) -> source partitions per combine vertex
        self.vids: list[list[int]] = []
        self.inputs_of: dict = {}    # vid -> [[(src_vid, src_port, edge_id), ...] per stage input]
        self.events = []
        self.compress = ctx.IntermediateDataCompressionScheme.value != 0
        self.output_gzip = ctx.OutputDataCompressionScheme.value != 0
        self._build()

    # ------------------------------------------------------------------ graph construction
    def _build(self):
        g = self.g
        for s in self.plan.stages:
            sid = g.add_stage(f"{s.id}:{s.name}", s.partitions, True, s.is_output)
            assert sid == s.id
            self.vids.append([g.add_vertex(sid, p) for p in range(s.partitions)])
        edge_count = 0
        for s in self.plan.stages:
            for p in range(s.partitions):
                dst = self.vids[s.id][p]
                lists = []
                for ii, si in enumerate(s.inputs):
                    src_stage = self.plan.stages[si.src]
                    lst = []
                    if si.kind == "pointwise":
                        pairs = [(self.vids[si.src][p], si.port)]
                    elif si.kind == "cross":
                        pairs = [(v, p) for v in self.vids[si.src]]
                    elif si.kind in ("merge", "broadcast"):
                        pairs = [(v, si.port) for v in self.vids[si.src]]
                    elif si.kind == "offset":
                        q = p - si.offset
                        pairs = [(self.vids[si.src][q], si.port)] if 0 <= q < src_stage.partitions else []
                    elif si.kind == "group" and getattr(si, "dynamic", False):
                        # dynamic aggregation: every combine vertex waits for all the partials; which
                        # of them it reads is decided from their sizes when it is scheduled
                        pairs = [(v, si.port) for v in self.vids[si.src]]
                    elif si.kind == "group":
                        pairs = [(self.vids[si.src][q], si.port)
                                 for q in range(p * si.group, min(src_stage.partitions, (p + 1) * si.group))]
                    else:
                        raise DryadLinqException(ErrorCode.Internal, f"unknown connection {si.kind}")
                    for src, port in pairs:
                        g.add_edge(src, port, dst, ii)
                        lst.append((src, port, edge_count))
                        edge_count += 1
                    lists.append(lst)
                self.inputs_of[dst] = lists
        # gang: members of a collective exchange (cross edges) must restart together on failure
        # in the GPU executor; the CPU executor's file channels do not need it.
        self.topology = json.loads(g.topology_json())

    # ------------------------------------------------------------------ channels
    def chan_path(self, vid, version, port):
        return os.path.join(self.job_dir, "ch", f"v{vid}.{version}.p{port}")

    def output_part_path(self, stage, partition, vid, version):
        uri = stage.output["uri"]
        scheme, path, _ = parse_uri(uri)
        if scheme in ("partfile", "file"):
            base = PF.default_base(path)
            os.makedirs(os.path.dirname(base), exist_ok=True)
            return PF.tmp_part_path(base, partition, vid, 0, version)
        return os.path.join(self.job_dir, "out", f"s{stage.id}.p{partition}.v{version}")

    def _dynamic_group(self, stage, ii, part):
        """Source partitions the combine vertex ``part`` of ``stage`` folds (runtime/aggmanager):
        decided once per stage input from the partials' sizes, then kept for re-executions."""
        key = (stage.id, ii)
        if key not in self.dyn_groups:
            from .aggmanager import assign_groups, parse_size
            si = stage.inputs[ii]
            sizes = [int(self.out_bytes.get(v, 0)) for v in self.vids[si.src]]
            props = getattr(self.ctx, "_props", {})
            thr = parse_size(props.get("AggregateThreshold") or (1 << 30))
            max_in = int(props.get("AggregationTreeMaxInputs") or 150)
            groups = assign_groups(sizes, stage.partitions, max_in, thr)
            self.dyn_groups[key] = groups
            self._event(dict(event="dynamic_aggregate", stage=f"{stage.id}:{stage.name}", threshold=thr,
                             partials=len(sizes), partial_bytes=sum(sizes),
                             groups=[len(x) for x in groups if x]))
        return set(self.dyn_groups[key][part])

    def command(self, vid, version):
        g = self.g
        sid = g.vertex_stage(vid)
        part = g.vertex_partition(vid)
        stage = self.plan.stages[sid]
        inputs = []
        for ii, lst in enumerate(self.inputs_of[vid]):
            si = stage.inputs[ii]
            if si.kind == "group" and getattr(si, "dynamic", False):
                chosen = self._dynamic_group(stage, ii, part)
                lst = [(src, port, e) for src, port, e in lst if g.vertex_partition(src) in chosen]
            inputs.append([(self.chan_path(src, g.completed_version(src), port), e) for src, port, e in lst])
        cmd = dict(job=self.job_dir, stage=sid, partition=part, vertex=vid, version=version, inputs=inputs,
                   outputs=[self.chan_path(vid, version, k) for k in range(stage.out_ports)],
                   faults=self.faults, compress=self.compress, output_gzip=self.output_gzip)
        if stage.is_output:
            cmd["output_part"] = self.output_part_path(stage, part, vid, version)
        return cmd

    def _dump_restart(self, cmd):
        """Restart record of one vertex attempt (reference DVertexPnController::DumpRestartCommand,
        dvertexpncontrol.cpp:348-736): the full command, so the vertex can be re-run on its own
        from its persisted input channels with ``python -m dryad_amd.runtime.vertexhost --cmd``."""
        d = os.path.join(self.job_dir, "log", "rerun")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"vertex-{cmd['vertex']}.{cmd['version']}.json"), "w") as f:
            json.dump(cmd, f, indent=1, default=str)

    def _inputs_complete(self, vid) -> bool:
        return all(self.g.completed_version(src) >= 0 for lst in self.inputs_of[vid] for src, _, _ in lst)

    # ------------------------------------------------------------------ main loop
    def _event(self, e: dict):
        self.events.append(e)
        if self.handle is not None:
            self.handle.events.append(e)

    def run(self):
        g = self.g
        t0 = time.time()
        now = lambda: time.time() - t0  # noqa: E731
        os.makedirs(os.path.join(self.job_dir, "ch"), exist_ok=True)
        os.makedirs(os.path.join(self.job_dir, "out"), exist_ok=True)
        self._check_outputs()
        g.start(now())
        running = {}          # (vid, version) -> slot
        pending = []          # ReadyItems waiting for a slot
        results = {}          # vid -> result of the winning version
        # event pump (DrMessagePump): results, the duplicate-check timer and a user cancel are
        # messages; the loop blocks in pump.wait() (GIL released) until one is due
        from ..jobinfo import MSG_CANCEL, MSG_DUPLICATES, MSG_RESULT
        pump = native_runtime().MessagePump()
        self.pump = pump
        self.pool.attach(pump, MSG_RESULT)
        if self.handle is not None:
            self.handle.pump = pump
        pump.post_after(int(self.DUPLICATE_CHECK_MS), MSG_DUPLICATES)
        try:
            while not g.done():
                if g.failed():
                    break
                if self.handle is not None and self.handle.cancelled:
                    g.abort("job cancelled by the user")
                    break
                pending.extend(g.take_ready(1 << 20, now()))
                still = []
                for it in pending:
                    if g.completed_version(it.vertex) >= 0 or not self._inputs_complete(it.vertex):
                        g.on_cancelled(it.vertex, it.version, now())   # stale: duplicate won / input invalidated
                        continue
                    slot = self.pool.acquire()
                    if slot is None:
                        still.append(it)
                        continue
                    cmd = self.command(it.vertex, it.version)
                    self._dump_restart(cmd)
                    g.on_running(it.vertex, it.version, slot, now())
                    self.pool.send(slot, cmd)
                    running[(it.vertex, it.version)] = slot
                pending = still
                if not running and not pending and not g.done():
                    if g.ready_count() == 0:
                        g.abort("deadlock: nothing runnable")
                        break
                    continue
                for kind, _ in pump.wait(-1 if running else 0):
                    if kind == MSG_DUPLICATES:
                        # duplicates are queued inside the JobGraph; take_ready hands them out
                        g.check_duplicates(now())
                        pump.post_after(int(self.DUPLICATE_CHECK_MS), MSG_DUPLICATES)
                for slot, res in self.pool.poll(0):
                    key = (res["vertex"], res["version"])
                    running.pop(key, None)
                    self.pool.release(slot)
                    self._handle_result(res, running, results, now)
                self.pool.rearm()
                self._drain_events()
            self._drain_events()
            if g.failed():
                for key, slot in list(running.items()):
                    self.pool.kill(slot)
                raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed, g.failure(),
                                            inner=getattr(self, "_last_exc", None))
            committed = self._commit(results)
            return dict(results=results, committed=committed, elapsed=time.time() - t0,
                        statistics=json.loads(g.statistics_json()))
        finally:
            for key, slot in list(running.items()):
                self.pool.kill(slot)
            self.pool.attach(None, MSG_RESULT)
            if self.handle is not None:
                self.handle.pump = None
            self.pump_stats = dict(posted=pump.posted(), delivered=pump.delivered())
            pump.close()

    def _handle_result(self, res, running, results, now):
        g = self.g
        v, ver = res["vertex"], res["version"]
        if res.get("lost"):
            res["error"] = res.get("error") or "vertex host process died"
        if res["ok"]:
            accepted, cancel = g.on_completed(v, ver, now(), int(res["bytes_read"]), int(res["bytes_written"]))
            if accepted:
                results[v] = res
                self.out_bytes[v] = int(res["bytes_written"])
            for cv, cver in cancel:
                slot = running.pop((cv, cver), None)
                if slot is not None:
                    self.pool.kill(slot)
                g.on_cancelled(cv, cver, now())
        else:
            if res.get("exc") is not None:
                self._last_exc = res["exc"]
            out = g.on_failed(v, ver, now(), int(res.get("bad_edge", -1)), str(res.get("error"))[:2000])
            for cv, cver in out.cancel:
                slot = running.pop((cv, cver), None)
                if slot is not None:
                    self.pool.kill(slot)
            log.info("vertex %d.%d failed: %s", v, ver, str(res.get("error")).splitlines()[0] if res.get("error") else "")

    def _drain_events(self):
        for e in self.g.drain_events():
            try:
                self._event(json.loads(e))
            except ValueError:
                pass

    # ------------------------------------------------------------------ outputs
    def _check_outputs(self):
        for s in self.plan.stages:
            if s.is_output:
                uri = s.output["uri"]
                p = provider_for(uri)
                if p.exists(uri):
                    if s.output.get("delete_if_exists") or s.output.get("temp"):
                        p.delete(uri)
                    else:
                        raise DryadLinqException(ErrorCode.JobToCreateTableFailed,
                                                 f"output {uri} already exists (use delete_if_exists=True)")

    def _commit(self, results):
        committed = {}
        for s in self.plan.stages:
            if not s.is_output:
                continue
            uri = s.output["uri"]
            scheme, path, _ = parse_uri(uri)
            vids = self.vids[s.id]
            res = [results[v] for v in vids]
            dtypes = {r["dtype"] for r in res if r.get("dtype")}
            fmts = {r["fmt"] for r in res if r.get("fmt")}
            dtype = s.output.get("dtype") or s.dtype
            if scheme in ("partfile", "file"):
                chosen = [self.output_part_path(s, p, v, self.g.completed_version(v)) for p, v in enumerate(vids)]
                base = PF.default_base(path)
                meta = PF.commit_parts(path, base, chosen)
                PF.cleanup_tmp(base)
                fmt = "pickle" if "pickle" in fmts else ("custom" if "custom" in fmts else "binary")
                if dtype is None or dtype == T.Pickle:
                    dtype = _resolve_dtype(dtypes, fmt)
                write_schema(path, dtype, fmt)
                committed[uri] = meta
            else:
                # any other provider (mem, hbm, text, user-registered): hand it the records
                from .worker import read_channel
                parts = []
                for p, v in enumerate(vids):
                    recs, _ = read_channel(self.output_part_path(s, p, v, self.g.completed_version(v)), -1)
                    parts.append(recs)
                prov = provider_for(uri)
                if not hasattr(prov, "write_table"):
                    raise DryadLinqException(ErrorCode.UnrecognizedDataSource, f"cannot write to {uri}")
                prov.write_table(uri, parts, dtype)
                committed[uri] = len(parts)
            qn = s.output.get("qnode")
            if qn is not None and qn.dtype is None:
                qn.dtype = dtype
        return committed


def _resolve_dtype(names, fmt):
    if fmt == "pickle":
        return T.Pickle
    if len(names) == 1:
        n = next(iter(names))
        if n in T.PRIMITIVES:
            return T.PRIMITIVES[n]
    return T.Pickle


def schema_path(meta_path: str) -> str:
    return meta_path + ".dryadtype"


_TRUSTED_PICKLED: set = set()


def pickled_table_trusted(meta_path: str) -> bool:
    """Opaque-record ("pickle" format) tables are only decoded when this process wrote them (the
    object executor's own temporaries) or the user opted in with DRYAD_TRUST_PICKLED_TABLES=1."""
    return os.path.abspath(meta_path) in _TRUSTED_PICKLED or os.environ.get("DRYAD_TRUST_PICKLED_TABLES") == "1"


def write_schema(meta_path: str, dtype, fmt: str, **extra):
    """Sidecar of a partfile table: record type and part format ("binary" DryadLinqBinary records,
    "pickle", or "rows" = raw fixed-width rows with ``stride`` / ``key_off`` / ``key_len``).
    Declarative JSON (types.dtype_to_json), so reading a foreign table's schema executes nothing;
    a type without a descriptor is stored as ``null`` (readers then infer from the records)."""
    try:
        d = T.dtype_to_json(dtype)
    except TypeError:
        d = None
    if fmt == "pickle":
        _TRUSTED_PICKLED.add(os.path.abspath(meta_path))
    with open(schema_path(meta_path), "w") as f:
        json.dump({"dtype": d, "format": fmt, **extra}, f)


def read_schema(meta_path: str):
    p = schema_path(meta_path)
    if not os.path.exists(p):
        return None
    with open(p, "rb") as f:
        raw = f.read()
    try:
        d = json.loads(raw.decode("utf-8"))
    except (UnicodeDecodeError, ValueError):
        log.warning("ignoring non-JSON schema sidecar %s (older pickled format is not loaded)", p)
        return None
    d["dtype"] = T.dtype_from_json(d.get("dtype"))
    return d
