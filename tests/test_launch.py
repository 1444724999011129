"""Native per-GPU launcher: env:// contract, SPMD job over gloo, gang failure handling."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launcher():
    from dryad_amd._build import build_launcher
    return str(build_launcher())


def test_launcher_sets_rank_env(tmp_path):
    script = tmp_path / "env.py"
    script.write_text("import os\nprint('R', os.environ['RANK'], os.environ['WORLD_SIZE'], os.environ['MASTER_ADDR'])\n")
    out = subprocess.run([_launcher(), "--gpus", "3", "--log-dir", str(tmp_path / "logs"), "--", sys.executable,
                          str(script)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    lines = sorted(open(tmp_path / "logs" / f"rank{r}.log").read().strip() for r in range(3))
    assert lines == [f"R {r} 3 127.0.0.1" for r in range(3)]


def test_launcher_stops_gang_when_a_rank_fails(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ['RANK'] == '1':
            sys.exit(3)
        time.sleep(60)
    """))
    out = subprocess.run([_launcher(), "--gpus", "3", "--grace-seconds", "2", "--", sys.executable, str(script)],
                         capture_output=True, text=True, timeout=40)
    assert out.returncode == 3
    assert "job failed: rank 1" in out.stderr


@pytest.mark.timeout(300)
def test_spmd_query_job_through_launcher(tmp_path):
    env = dict(os.environ, SPMD_DEVICE="cpu", PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "dryad_amd.launch", "--gpus", "2", "--master-port", "29617",
                          os.path.join(ROOT, "tests", "dist", "spmd_queries.py")],
                         capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "SPMD_OK 2" in out.stdout


@pytest.mark.timeout(300)
def test_gang_relaunch_resumes_after_a_lost_rank(tmp_path):
    """Rank 1 is SIGKILLed mid-stage (a real lost process): dryad-launch stops the gang, starts a
    fresh one (new processes, new rendezvous port), and the job resumes from the persisted stage
    outputs: oracle-equal result, a gang_relaunch event in the job's events.jsonl, stage 0 not run
    again (a stage_resumed event) and the relaunch in the launcher's own log."""
    import json
    env = dict(os.environ, SPMD_DEVICE="cpu", PYTHONPATH=ROOT, DRYAD_HOME=str(tmp_path / "home"))
    logs = tmp_path / "logs"
    # no --checkpoint-dir: a relaunching launcher persists to its own directory under /dev/shm
    out = subprocess.run([_launcher(), "--gpus", "2", "--master-port", "29641", "--grace-seconds", "3",
                          "--max-restarts", "2", "--log-dir", str(logs),
                          "--", sys.executable, os.path.join(ROOT, "tests", "dist", "gang_relaunch_job.py")],
                         capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:] + open(logs / "rank0.log").read()[-2000:]
    rank0 = open(logs / "rank0.e1.log").read()
    line = next(ln for ln in rank0.splitlines() if ln.startswith("{"))
    rep = json.loads(line)
    assert rep["ok"] and rep["n"] > 0 and rep["epoch"] == 1, rep
    assert ["resumed", rep["stages"][0]] in rep["recovery"], rep["recovery"]
    evs = [json.loads(x) for x in open(os.path.join(rep["job_dir"], "log", "events.jsonl"))]
    kinds = [e.get("ev") for e in evs]
    assert "gang_relaunch" in kinds and "stage_resumed" in kinds, kinds
    ck = next(e for e in evs if e.get("ev") == "gang_relaunch")["checkpoint"]
    assert ck.startswith("/dev/shm/dryad-ckpt-"), ck
    assert not os.path.exists("/".join(ck.split("/")[:4])), ck     # the launcher removed its directory
    assert "stage_persisted" in kinds, kinds
    relaunch = next(e for e in evs if e.get("ev") == "gang_relaunch")
    assert relaunch["epoch"] == 1 and "rank 1 lost" in relaunch["reason"], relaunch
    launcher = [json.loads(x) for x in open(logs / "launcher.jsonl")]
    assert launcher[0]["ev"] == "gang_relaunch" and launcher[0]["rank"] == 1 and launcher[0]["status"] == 128 + 9
    assert launcher[-1]["ev"] == "job_complete"
    assert "(signal)" in out.stderr


def test_launcher_does_not_relaunch_a_deterministic_failure(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '0' else 0)\n")
    out = subprocess.run([_launcher(), "--gpus", "2", "--max-restarts", "3", "--", sys.executable, str(script)],
                         capture_output=True, text=True, timeout=40)
    assert out.returncode == 3 and "epoch 1" not in out.stderr, out.stderr


def test_launcher_checkpoint_dir_is_launcher_owned(tmp_path):
    """--checkpoint-dir names a PARENT: the ranks get <dir>/dryad-ckpt-<launcher pid>, which the
    launcher removes when it exits; the user's own files under <dir> are never touched."""
    d = tmp_path / "data"
    d.mkdir()
    (d / "keep.txt").write_text("user data")
    script = tmp_path / "ck.py"
    script.write_text("import os\nc = os.environ['DRYAD_CHECKPOINT_DIR']\nassert os.path.isdir(c), c\n"
                      "open(os.path.join(c, 'x' + os.environ['RANK']), 'w').write('1')\nprint(c)\n")
    out = subprocess.run([_launcher(), "--gpus", "2", "--checkpoint-dir", str(d), "--log-dir", str(tmp_path / "logs"),
                          "--", sys.executable, str(script)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    owned = open(tmp_path / "logs" / "rank0.log").read().strip()
    assert os.path.dirname(owned) == str(d) and os.path.basename(owned).startswith("dryad-ckpt-"), owned
    assert sorted(os.listdir(d)) == ["keep.txt"] and (d / "keep.txt").read_text() == "user data"
    bad = subprocess.run([_launcher(), "--gpus", "1", "--checkpoint-dir", str(d / "keep.txt"), "--", sys.executable,
                          "-c", "pass"], capture_output=True, text=True, timeout=60)
    assert bad.returncode == 2 and (d / "keep.txt").exists()
