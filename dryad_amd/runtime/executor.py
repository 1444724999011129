"""Job executors: compile queries, run the job, expose results.

* ``LocalExecutor`` — the LocalJobSubmission analog (LinqToDryad/LocalJobSubmission.cs:97-373):
  a job directory ``<home>/LocalJobs/<n>/`` with the plan, channels and logs
  (``log/events.jsonl`` Calypso-style, ``log/error.txt`` on failure, ``statistics.json``),
  the job manager in the client process and N vertex-host processes.
* ``GpuExecutor`` (dryad_amd/runtime/gpu_executor.py) — SPMD over MI355X ranks.
"""
from __future__ import annotations

import itertools
import json
import os
import shutil
import threading
import time

from ..compiler.planner import compile_queries
from ..errors import DryadLinqException
from ..io.providers import provider_for
from ..query import Query
from ..utils.log import get_logger
from .jobmanager import JobRunner
from .pool import ProcessPool, ThreadPool

log = get_logger("executor")


def make_executor(ctx):
    from ..context import PlatformKind
    if ctx.PlatformKind == PlatformKind.GPU:
        from .gpu_executor import GpuExecutor
        return GpuExecutor(ctx)
    return LocalExecutor(ctx)


def dryad_home(ctx) -> str:
    h = ctx.DryadHomeDirectory or os.environ.get("DRYAD_HOME")
    if not h:
        h = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"dryad-home-{os.getuid()}")
    os.makedirs(h, exist_ok=True)
    return h


class _BaseExecutor:
    def enumerate(self, q: Query) -> list:
        node = q.node
        if node.op == "ToStore":
            if not node.args.get("_executed"):
                self.ctx.SubmitAndWait(q)
            uri = node.args["uri"]
            return list(provider_for(uri).read_all(uri, node.dtype))
        tmp = self.ctx.MakeTemporaryStreamUri()
        st = q.ToStore(tmp)
        st.node.args["_temp"] = True
        self.run_job([st], None)
        p = provider_for(tmp)
        try:
            return list(p.read_all(tmp, st.node.dtype))
        finally:
            try:
                p.delete(tmp)
            except Exception:
                pass

    def _enter_job_thread(self):
        """Per-thread setup of a job thread (the GPU executor binds it to its rank's device)."""

    def submit(self, outs, handle):
        handle.t_submit = time.perf_counter()

        def body():
            try:
                self._enter_job_thread()
            except BaseException as e:  # noqa: BLE001
                handle.finish(False, e)
                return
            handle.set_running()
            try:
                r = self.run_job(outs, handle)
                handle.finish(True, result=r)
            except BaseException as e:  # noqa: BLE001
                handle.finish(False, e)
        t = threading.Thread(target=body, daemon=True, name=f"dryad-job-{handle.job_id}")
        handle.thread = t
        t.start()


class LocalExecutor(_BaseExecutor):
    def __init__(self, ctx):
        self.ctx = ctx
        n = int(ctx.NumProcesses or 2)
        mode = os.environ.get("DRYAD_POOL", ctx._props.get("PoolKind", "process"))
        self.thread_pool = mode == "thread"
        self.pool = ThreadPool(n) if self.thread_pool else ProcessPool(n)
        self.home = dryad_home(ctx)
        self._seq = itertools.count(1)
        self._lock = threading.Lock()
        self.last_job_dir = None
        self.last_result = None

    def _new_job_dir(self) -> str:
        root = os.path.join(self.home, "LocalJobs")
        os.makedirs(root, exist_ok=True)
        while True:
            d = os.path.join(root, f"{os.getpid()}-{int(time.time() * 1000) % 10**9}-{next(self._seq)}")
            if not os.path.exists(d):
                os.makedirs(os.path.join(d, "log"))
                return d

    def run_job(self, outs, handle):
        import cloudpickle
        with self._lock:
            plan = compile_queries(self.ctx, outs)
            job_dir = self._new_job_dir()
            self.last_job_dir = job_dir
            with open(os.path.join(job_dir, "plan.pkl"), "wb") as f:
                cloudpickle.dump(plan, f)
            with open(os.path.join(job_dir, "plan.json"), "w") as f:
                f.write(plan.dumps())
            with open(os.path.join(job_dir, "QueryPlan.xml"), "w") as f:   # the reference job directory's plan
                f.write(plan.to_xml())
            with open(os.path.join(job_dir, "QueryGraph.txt"), "w") as f:
                f.write(plan.explain())
            if self.thread_pool:
                self.pool.register_plan(job_dir, plan)
            faults = self.ctx._props.get("FaultInjection") or _env_faults()
            runner = JobRunner(self.ctx, plan, self.pool, job_dir, handle, faults)
            ok = False
            try:
                res = runner.run()
                ok = True
                for s in plan.stages:
                    if s.is_output and s.output.get("qnode") is not None:
                        s.output["qnode"].args["_executed"] = True
                with open(os.path.join(job_dir, "statistics.json"), "w") as f:
                    json.dump(res["statistics"], f, indent=1)
                self.last_result = res
                return res
            except BaseException as e:
                with open(os.path.join(job_dir, "log", "error.txt"), "w") as f:
                    f.write(str(e))
                raise
            finally:
                with open(os.path.join(job_dir, "log", "events.jsonl"), "w") as f:
                    for e in runner.events:
                        f.write(json.dumps(e) + "\n")
                if ok and not self.ctx._props.get("KeepJobDirectories"):
                    shutil.rmtree(os.path.join(job_dir, "ch"), ignore_errors=True)
                    shutil.rmtree(os.path.join(job_dir, "out"), ignore_errors=True)

    def close(self):
        self.pool.close()


def _env_faults():
    """DRYAD_FAULT_INJECT="stage:partition:version:kind,..." (any field may be '*')."""
    spec = os.environ.get("DRYAD_FAULT_INJECT")
    if not spec:
        return []
    out = []
    for item in spec.split(","):
        parts = (item.split(":") + ["*", "*", "*", "fail"])[:4]
        st, p, v, kind = parts
        conv = lambda x: None if x == "*" else (int(x) if x.lstrip("-").isdigit() else x)  # noqa: E731
        out.append(dict(stage=conv(st), partition=conv(p), version=conv(v), kind=kind))
    return out
