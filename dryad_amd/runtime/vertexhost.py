"""Vertex host process entry point (the VertexHost.exe analog).

    python -m dryad_amd.runtime.vertexhost --address <unix socket> --slot <i> --authkey <hex>

Launched by the ProcessPool as an independent program (never a fork of the client, so user
``__main__`` modules are not re-imported), it connects back to the job manager and serves vertex
commands until told to stop (reference: VertexHostMain/Program.cs -> vertexHost.cpp:252-364).
"""
from __future__ import annotations

import argparse
import os
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--slot", type=int, required=True)
    ap.add_argument("--authkey", required=True)
    a = ap.parse_args(argv)
    from multiprocessing.connection import Client
    from .worker import worker_main
    conn = Client(a.address, family="AF_UNIX", authkey=bytes.fromhex(a.authkey))
    worker_main(conn, a.slot)


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if root not in sys.path:
        sys.path.insert(0, root)
    main()
