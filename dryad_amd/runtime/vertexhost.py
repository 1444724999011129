"""Vertex host process entry point (the VertexHost.exe analog).

    python -m dryad_amd.runtime.vertexhost --address <unix socket> --slot <i> --authkey <hex>
    python -m dryad_amd.runtime.vertexhost --cmd <job>/log/rerun/vertex-V.v.json [--out DIR]

Launched by the ProcessPool as an independent program (never a fork of the client, so user
``__main__`` modules are not re-imported), it connects back to the job manager and serves vertex
commands until told to stop (reference: VertexHostMain/Program.cs -> vertexHost.cpp:252-364).
"""
from __future__ import annotations

import argparse
import os
import sys


def run_cmd(path: str, out_dir: str | None = None, keep_faults: bool = False) -> dict:
    """Standalone controller (reference DVertexCmdLineController, dvertexcmdlinecontrol.cpp:926-1030):
    re-run one vertex from the restart record a job wrote for it (``log/rerun/vertex-V.v.json``),
    reading its persisted input channels, writing its outputs under ``out_dir`` (default
    ``<job>/rerun-out``) so the job's own files are untouched.  Injected faults are dropped unless
    ``keep_faults``."""
    import json
    from .worker import execute_vertex
    with open(path) as f:
        cmd = json.load(f)
    out_dir = out_dir or os.path.join(cmd["job"], "rerun-out")
    os.makedirs(out_dir, exist_ok=True)
    tag = f"v{cmd['vertex']}.{cmd['version']}"
    cmd["outputs"] = [os.path.join(out_dir, f"{tag}.p{k}") for k in range(len(cmd["outputs"]))]
    if "output_part" in cmd:
        cmd["output_part"] = os.path.join(out_dir, f"{tag}.part")
    if not keep_faults:
        cmd["faults"] = []
    res = execute_vertex(cmd)
    res.pop("exc", None)
    res["outputs"] = cmd["outputs"] + ([cmd["output_part"]] if "output_part" in cmd else [])
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--address")
    ap.add_argument("--slot", type=int)
    ap.add_argument("--authkey")
    ap.add_argument("--cmd", help="re-run one vertex from its restart record and exit")
    ap.add_argument("--out", default=None)
    ap.add_argument("--keep-faults", action="store_true")
    a = ap.parse_args(argv)
    if a.cmd:
        import json
        res = run_cmd(a.cmd, a.out, a.keep_faults)
        print(json.dumps(res, default=str))
        return 0 if res.get("ok") else 1
    if a.address is None or a.slot is None or a.authkey is None:
        ap.error("--address, --slot and --authkey are required (or --cmd)")
    from multiprocessing.connection import Client
    from .worker import worker_main
    conn = Client(a.address, family="AF_UNIX", authkey=bytes.fromhex(a.authkey))
    worker_main(conn, a.slot)


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if root not in sys.path:
        sys.path.insert(0, root)
    sys.exit(main() or 0)
