"""Standalone vertex replay from restart records (reference DumpRestartCommand + the --cmd vertex
controller) and the job browser's failure diagnosis (Diagnosis.cs), on both executors (CPU)."""
import glob
import json
import os
import subprocess
import sys

import pytest

import dryad_amd as D
from dryad_amd.errors import DryadLinqJobException
from dryad_amd.tools import jobbrowser as JB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAIRS = [(i % 17, i) for i in range(3000)]


def _query(c):
    return c.FromEnumerable(PAIRS).GroupBy(lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1])))


def test_process_executor_restart_record_replays_failed_vertex(tmp_path):
    c = D.DryadLinqContext(2)
    c.PartitionCount = 2
    c.DryadHomeDirectory = str(tmp_path)
    c.FaultInjection = [dict(stage=None, partition=1, version=None, kind="fail")]     # fails every attempt
    with pytest.raises(DryadLinqJobException):
        list(_query(c))
    job = c._get_executor().last_job_dir
    recs = sorted(glob.glob(os.path.join(job, "log", "rerun", "vertex-*.json")))
    assert recs
    diag = JB.diagnose(JB.load(job))
    text = "\n".join(diag)
    assert "deterministic" in text and "vertexhost --cmd" in text, text
    failing = next(r for r in recs if json.load(open(r))["partition"] == 1)
    out = subprocess.run([sys.executable, "-m", "dryad_amd.runtime.vertexhost", "--cmd", failing,
                          "--out", str(tmp_path / "replay")], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["ok"] and all(os.path.exists(p) for p in res["outputs"])
    keep = subprocess.run([sys.executable, "-m", "dryad_amd.runtime.vertexhost", "--cmd", failing, "--keep-faults",
                           "--out", str(tmp_path / "replay2")], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert keep.returncode == 1                  # the injected fault reproduces the failure


def test_gpu_executor_restart_record_replays_on_cpu(tmp_path):
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 2
    c.DryadHomeDirectory = str(tmp_path)
    c.FaultInjection = [dict(stage=None, partition=0, version=None, kind="crash")]
    with pytest.raises(DryadLinqJobException):
        list(_query(c))
    job = c._get_executor().last_job_dir
    dirs = sorted(d for d in glob.glob(os.path.join(job, "log", "rerun", "vertex-*")) if os.path.isdir(d))
    assert dirs
    text = "\n".join(JB.diagnose(JB.load(job)))
    assert "dryad_amd.tools.replay" in text and "failed 6x" in text, text
    from dryad_amd.tools import replay as RP
    ok, out = RP.replay(dirs[0], "cpu")
    assert ok, out
    r = subprocess.run([sys.executable, "-m", "dryad_amd.tools.replay", dirs[0], "--device", "cpu"],
                       capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0 and "vertex completed" in r.stdout, r.stdout + r.stderr
