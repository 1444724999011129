"""Job browser for LocalJobs directories (reference JobBrowser, §5.1: plan, stage statistics,
vertex schedule, failure diagnosis, and a timeline view).

    python -m dryad_amd.tools.jobbrowser                # newest job under $DRYAD_HOME/LocalJobs
    python -m dryad_amd.tools.jobbrowser JOB_DIR [--vertices] [--chrome-trace out.json]

A job directory holds ``plan.json`` / ``QueryGraph.txt`` (explain), ``log/events.jsonl``
(Calypso-style vertex state transitions from the native job graph), ``statistics.json`` (per
stage: executions, failures, mean/max running time, outlier threshold, bytes) and
``log/error.txt`` on failure.  ``--chrome-trace`` writes the vertex executions as a Chrome /
Perfetto trace (one track per worker).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics as stats
import sys


def newest_job(home: str | None = None) -> str | None:
    home = home or os.environ.get("DRYAD_HOME") or os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                                               f"dryad-home-{os.getuid()}")
    jobs = glob.glob(os.path.join(home, "LocalJobs", "*"))
    return max(jobs, key=os.path.getmtime) if jobs else None


def load(job_dir: str) -> dict:
    import sys
    if "dryad_amd.runtime.gpu_executor" in sys.modules:      # in-process: queued GPU job-dir writes
        sys.modules["dryad_amd.runtime.gpu_executor"].flush_job_dirs()
    j = {"dir": job_dir, "events": [], "stats": {}, "explain": "", "error": None}
    ev = os.path.join(job_dir, "log", "events.jsonl")
    if os.path.exists(ev):
        with open(ev) as f:
            j["events"] = [json.loads(x) for x in f if x.strip()]
    st = os.path.join(job_dir, "statistics.json")
    if os.path.exists(st):
        with open(st) as f:
            j["stats"] = json.load(f)
    ex = os.path.join(job_dir, "QueryGraph.txt")
    if os.path.exists(ex):
        with open(ex) as f:
            j["explain"] = f.read()
    er = os.path.join(job_dir, "log", "error.txt")
    if os.path.exists(er):
        with open(er) as f:
            j["error"] = f.read()
    return j


def executions(events: list) -> list:
    """One record per (vertex, version) run: start, end, state, worker, stage, partition."""
    runs = {}
    for e in events:
        if e.get("ev") != "vertex":
            continue
        k = (e["vertex"], e.get("version", 0))
        r = runs.setdefault(k, dict(vertex=e["vertex"], version=e.get("version", 0), stage=e.get("stage"),
                                    partition=e.get("partition"), start=None, end=None, state=None, worker=None,
                                    duplicate=False))
        if e["state"] == "Running":
            r["start"], r["worker"] = e["t"], e.get("worker")
        elif e["state"] in ("Completed", "Failed", "Canceled", "Cancelled"):
            r["end"], r["state"] = e["t"], e["state"]
            if "error" in e:
                r["error"] = e["error"]
        if e.get("duplicate"):
            r["duplicate"] = True
    return sorted(runs.values(), key=lambda r: (r["start"] if r["start"] is not None else 1e30, r["vertex"]))


# failure classes (JobBrowser Diagnosis.cs:36-929: vertex failure diagnosis, deterministic input
# failures, read failures per producer, aborts after too many failures, serialization errors)
_CLASSES = [
    ("out of memory", ("out of memory", "hipErrorOutOfMemory", "OutOfMemory", "FailedToAllocateNewNativeBuffer"),
     "a vertex ran out of GPU memory: raise PartitionCount, lower HbmBudgetBytes, or let OrderBy go "
     "out of core (ExternalSort=True)"),
    ("host fallback refused", ("HostFallbackMaxBytes",),
     "an operator could not run on the device and its input was too large for the host path: rewrite the "
     "lambda with traceable column arithmetic or set AllowHostFallback=True"),
    ("serialization", ("FailedToDeserialize", "UnpicklingError", "PicklingError", "GeneralSerializeFailure",
                       "cannot serialize", "not serializable"),
     "records could not be (de)serialized: check the record type / custom serializer"),
    ("read failure", ("read error", "ChannelReadError", "ChannelReadFailed", "failed to read"),
     "a vertex could not read an input channel: the producer was re-executed"),
    ("collective / rank failure", ("NCCL", "RCCL", "ProcessGroup", "Watchdog", "timed out"),
     "a collective exchange failed or timed out: a rank died or stalled (see the other ranks' logs)"),
    ("user code exception", ("Error", "Exception"), "an exception was raised by a user lambda or operator"),
]


def _classify(err: str):
    for name, pats, advice in _CLASSES:
        if any(p in err for p in pats):
            return name, advice
    return "unknown", ""


def diagnose(job: dict) -> list:
    """Failure / straggler findings (JobBrowser Diagnosis.cs analogue), most important first:
    the job abort reason, per failing vertex its failure class and whether it is deterministic
    (every attempt failed the same way = a bug, not a transient fault), read failures grouped by
    the blamed producer, recovery actions, stragglers, and the restart records to replay."""
    out = []
    err = (job["error"] or "").strip()
    if err:
        out.append(f"job failed: {err[:500]}")
        if "failed" in err and "times" in err:
            out.append("  the job was aborted because one vertex exhausted MaxVertexFailures (see below)")
        cls, advice = _classify(err)
        if advice:
            out.append(f"  class: {cls}: {advice}")
    runs = executions(job["events"])
    failed = [r for r in runs if r["state"] == "Failed"]
    by_vertex = {}
    for r in failed:
        by_vertex.setdefault((r["vertex"], r["stage"], r["partition"]), []).append(r)
    for (v, st, p), rs in sorted(by_vertex.items(), key=lambda kv: -len(kv[1])):
        errs = [x.get("error", "?") for x in rs]
        cls, advice = _classify(errs[-1])
        det = len(rs) > 1 and len({e.split(" v")[0] for e in errs}) == 1
        out.append(f"vertex {v} ({st}[{p}]) failed {len(rs)}x [{cls}]"
                   + (" - deterministic (identical error on every attempt)" if det else "") + f": {errs[-1][:300]}")
        if advice:
            out.append(f"  {advice}")
    reads = {}
    for e in job["events"]:
        if e.get("ev") == "vertex" and e.get("state") == "Invalidated":
            reads.setdefault((e.get("stage"), e.get("partition")), 0)
            reads[(e.get("stage"), e.get("partition"))] += 1
    for (st, p), n in reads.items():
        out.append(f"read failures blamed producer {st}[{p}] {n}x: it was invalidated and re-executed")
    rec = job["stats"].get("recovery") if isinstance(job.get("stats"), dict) else None
    if rec:
        kinds = {}
        for r in rec:
            kinds[r[0]] = kinds.get(r[0], 0) + 1
        out.append("recovery actions: " + ", ".join(f"{k} x{n}" for k, n in sorted(kinds.items())))
    by_stage = {}
    for r in runs:
        if r["start"] is not None and r["end"] is not None and r["state"] == "Completed":
            by_stage.setdefault(r["stage"], []).append(r)
    for st, rs in by_stage.items():
        if len(rs) < 3:
            continue
        med = stats.median(x["end"] - x["start"] for x in rs)
        for x in rs:
            d = x["end"] - x["start"]
            if med > 0 and d > 3 * med and d > 0.05:
                out.append(f"straggler: {st}[{x['partition']}] took {d:.3f}s (stage median {med:.3f}s)")
    reexec = {r["vertex"] for r in runs if r["version"] > 0}
    if reexec:
        out.append(f"{len(reexec)} vertices were re-executed (versions > 0)")
    rr = sorted(glob.glob(os.path.join(job["dir"], "log", "rerun", "vertex-*")))
    gpu = [x for x in rr if os.path.isdir(x)]
    if gpu:
        out.append(f"{len(gpu)} failed GPU vertex attempts can be replayed: python -m dryad_amd.tools.replay {gpu[0]}")
    elif failed and rr:
        v = failed[-1]
        cand = os.path.join(job["dir"], "log", "rerun", f"vertex-{v['vertex']}.{v['version']}.json")
        if os.path.exists(cand):
            out.append(f"replay the failed vertex: python -m dryad_amd.runtime.vertexhost --cmd {cand}")
    return out


def chrome_trace(job: dict) -> dict:
    evs = []
    for r in executions(job["events"]):
        if r["start"] is None or r["end"] is None:
            continue
        evs.append(dict(name=f"{r['stage']}[{r['partition']}] v{r['version']}", ph="X", ts=r["start"] * 1e6,
                        dur=(r["end"] - r["start"]) * 1e6, pid=0, tid=r["worker"] if r["worker"] is not None else -1,
                        args=dict(state=r["state"], vertex=r["vertex"])))
    return {"traceEvents": evs, "displayTimeUnit": "ms"}


def render(job: dict, show_vertices: bool = False) -> str:
    L = [f"job {job['dir']}"]
    if job["explain"]:
        L += ["", "plan:", job["explain"].rstrip()]
    st = job["stats"]
    if st:
        L += ["", "stages:"]
        for s in st.get("stages", []):
            L.append(f"  {s.get('name', '?'):40s} parts={s.get('partitions', '?'):>4} exec={s.get('executions', '?'):>4}"
                     f" fail={s.get('failures', 0):>2} mean={s.get('mean_s', 0):.4f}s max={s.get('max_s', 0):.4f}s"
                     f" read={s.get('bytes_read', 0)} written={s.get('bytes_written', 0)}")
        if st.get("stage_seconds"):
            L += ["", "stage wall time (GPU executor):"]
            for k, v in st["stage_seconds"].items():
                L.append(f"  {k:48s} {v * 1e3:10.2f} ms")
        if st.get("host_fallbacks"):
            L += ["", "operators that ran on the host:"] + [f"  {x}" for x in st["host_fallbacks"]]
    if show_vertices:
        L += ["", "vertex executions:"]
        for r in executions(job["events"]):
            d = (r["end"] - r["start"]) if r["start"] is not None and r["end"] is not None else None
            L.append(f"  v{r['vertex']:<5} {str(r['stage']):36s} p{r['partition']!s:<4} ver={r['version']} "
                     f"worker={r['worker']!s:<3} {r['state']!s:10s} {'' if d is None else f'{d:.4f}s'}")
    diag = diagnose(job)
    L += ["", "diagnosis:"] + ([f"  {x}" for x in diag] if diag else ["  no failures or stragglers"])
    return "\n".join(L)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m dryad_amd.tools.jobbrowser")
    ap.add_argument("job_dir", nargs="?")
    ap.add_argument("--vertices", action="store_true")
    ap.add_argument("--chrome-trace", default=None)
    a = ap.parse_args(argv)
    d = a.job_dir or newest_job()
    if not d or not os.path.isdir(d):
        print("no job directory found", file=sys.stderr)
        return 1
    job = load(d)
    print(render(job, a.vertices))
    if a.chrome_trace:
        with open(a.chrome_trace, "w") as f:
            json.dump(chrome_trace(job), f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
