"""Shared plumbing for the secondary benchmark configs of BASELINE.json (one process per GPU,
launched directly for 1 GPU or by torch.distributed.run for N; rank 0 prints one JSON line)."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def world():
    import torch
    from dryad_amd.parallel.comm import init_world
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    return init_world(device=dev)


def timed(world, fn):
    """Run fn between barriers + device syncs; returns max-over-ranks seconds."""
    import torch
    import torch.distributed as dist
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    if world.size > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    out = fn()
    sync()
    if world.size > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world.size > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=world.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, out


def report(world, rec: dict):
    if world.rank == 0:
        print(json.dumps(rec), flush=True)
