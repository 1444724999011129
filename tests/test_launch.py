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
