"""Job browser over LocalJobs directories: plan/stats rendering, failure diagnosis, trace export."""
import json

import dryad_amd as D
from dryad_amd.tools import jobbrowser as JB


def test_jobbrowser_renders_job_and_diagnoses_reexecution(tmp_path):
    c = D.DryadLinqContext(2)
    c.DryadHomeDirectory = str(tmp_path)
    c.FaultInjection = [dict(stage=0, partition=1, version=0, kind="fail")]
    assert sorted(c.FromEnumerable(list(range(200))).Select(lambda x: x % 11).Distinct()) == list(range(11))
    d = c._get_executor().last_job_dir
    job = JB.load(d)
    txt = JB.render(job, show_vertices=True)
    assert "stages:" in txt and "vertex executions:" in txt
    diag = JB.diagnose(job)
    assert any("failed" in x for x in diag) and any("re-executed" in x for x in diag)
    tr = JB.chrome_trace(job)
    assert tr["traceEvents"] and all(e["ph"] == "X" for e in tr["traceEvents"])
    out = tmp_path / "t.json"
    assert JB.main([d, "--chrome-trace", str(out)]) == 0
    assert json.loads(out.read_text())["traceEvents"]
