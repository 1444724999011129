"""``python -m dryad_amd.launch --gpus N script.py [args]`` — one SPMD worker per GPU.

Front end of the native launcher (csrc/launcher/dryad_launch.cpp, built into
dryad_amd/_native/dryad-launch): it sets the torch.distributed env:// variables for each rank
(MASTER_ADDR=127.0.0.1), runs every rank in its own process group, and stops the whole gang when
one rank fails; with ``--max-restarts K`` a gang that lost a rank process is relaunched as new
processes and resumes from the persisted stage outputs.  The job script simply builds a ``DryadLinqContext(platform="gpu")``; the GPU
executor picks up RANK / WORLD_SIZE and initialises RCCL.
"""
from __future__ import annotations

import argparse
import subprocess
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m dryad_amd.launch")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--master-port", type=int, default=29511)
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--grace-seconds", type=int, default=10)
    ap.add_argument("--max-restarts", type=int, default=0,
                    help="relaunch the whole gang (new processes) up to K times when a rank process is lost; "
                         "the job resumes from persisted stage outputs (runtime/checkpoint.py)")
    ap.add_argument("--checkpoint-dir", default=None, help="where stage outputs are persisted for a relaunch")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    from ._build import LAUNCHER, build_launcher
    if not LAUNCHER.exists():
        build_launcher()
    cmd = [str(LAUNCHER), "--gpus", str(a.gpus), "--master-port", str(a.master_port),
           "--grace-seconds", str(a.grace_seconds)]
    if a.log_dir:
        cmd += ["--log-dir", a.log_dir]
    if a.max_restarts:
        cmd += ["--max-restarts", str(a.max_restarts)]
    if a.checkpoint_dir:
        cmd += ["--checkpoint-dir", a.checkpoint_dir]
    prog = [sys.executable, a.script] if a.script.endswith(".py") else [a.script]
    # the launcher is a child, not an exec replacement: this process never touched the GPU either way
    return subprocess.call(cmd + ["--"] + prog + list(a.args))


if __name__ == "__main__":
    sys.exit(main())
