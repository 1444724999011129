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


def diagnose(job: dict) -> list:
    """Failure / straggler findings (JobBrowser Diagnosis.cs analogue)."""
    out = []
    if job["error"]:
        out.append(f"job failed: {job['error'].strip()[:500]}")
    runs = executions(job["events"])
    failed = [r for r in runs if r["state"] == "Failed"]
    for r in failed:
        out.append(f"vertex {r['vertex']} ({r['stage']}[{r['partition']}]) v{r['version']} failed on worker "
                   f"{r['worker']}: {r.get('error', '?')}")
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
