"""Process-group management: one process per GPU, RCCL over xGMI (``torch.distributed`` backend
``"nccl"`` is RCCL on ROCm), ``gloo`` for CPU runs and tests.

This replaces the reference's whole cluster plane (Peloponnese process manager, YARN AM,
ProcessService HTTP mailboxes: SURVEY §2.4) for the single-node MI355X target: the set of
"computers" is the set of ranks, membership is fixed for a job, and all data-plane transfers go
through collectives on one communicator.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class World:
    rank: int = 0
    size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None
    # a one-rank world whose exchanges still go through the collectives (a one-rank RCCL
    # communicator: tests run the multi-rank code paths against real RCCL on a one-GPU box)
    force_collectives: bool = False

    @property
    def collective(self) -> bool:
        """Data movement goes through the process group (several ranks, or force_collectives)."""
        return self.size > 1 or self.force_collectives

    @property
    def distributed(self) -> bool:
        return self.size > 1 and dist.is_available() and dist.is_initialized()

    def barrier(self):
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


_WORLD: World | None = None


def env_world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


# Collective timeout: a rank that dies mid-exchange is detected by its peers' RCCL watchdog within
# this bound (the reference's process abort timeout is 30 s, DrGraphParameters.cpp:51; a 125 GB
# all-to-all-v round takes seconds, so the bound is minutes, not the 30 of torch's default).
COLLECTIVE_TIMEOUT_S = 300


def init_world(device: str | None = None, backend: str | None = None, timeout_s: int = COLLECTIVE_TIMEOUT_S) -> World:
    """Initialise (idempotently) the job's process group from torchrun-style env vars.

    ``device``: "cuda" / "cpu" / None (cuda if available).  The backend defaults to nccl (RCCL) for
    GPU ranks and gloo for CPU ranks.  RCCL runs with asynchronous error handling in tear-down mode:
    a collective error or timeout aborts the communicator and ends the rank, so the launcher
    (dryad-launch / torchrun) stops the whole gang instead of leaving the peers blocked."""
    global _WORLD
    if _WORLD is not None:
        return _WORLD
    size = env_world_size()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_cuda = (device == "cuda") or (device is None and torch.cuda.is_available())
    # DRYAD_DIST_BACKEND=gloo with GPU ranks: collectives staged through host memory.  Lets
    # several ranks share one GPU (RCCL needs distinct devices) so the multi-rank GPU data path
    # can be tested on a single-GPU box.
    be = backend or os.environ.get("DRYAD_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    if use_cuda:
        idx = local_rank
        if be != "nccl":
            idx = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
        if os.environ.get("DRYAD_NUMA_BIND", "1") == "1":
            # one rank per GPU: threads and pinned host buffers on the GPU's NUMA node
            from .affinity import bind_to_gpu
            bind_to_gpu(idx)
    else:
        dev = torch.device("cpu")
    if size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kwargs = dict(backend=be, rank=rank, world_size=size, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kwargs["device_id"] = dev
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group(**kwargs)
        if be == "nccl":
            warm_collectives(dev, size)
    _WORLD = World(rank=rank, size=size, local_rank=local_rank, device=dev, backend=be if size > 1 else None)
    return _WORLD


def warm_collectives(dev: torch.device, size: int):
    """One small all-to-all, all-gather and all-reduce right after the communicator is created:
    RCCL connects its point-to-point channels (and allocates their buffers) on a peer's first
    send / receive, so this happens before a job fills HBM with its working set, not inside the
    first 100 GB exchange with a few GB left."""
    x = torch.arange(size, dtype=torch.int32, device=dev)
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    g = torch.empty(size, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(g, x[:1].contiguous())
    dist.all_reduce(y)
    torch.cuda.synchronize(dev)


def init_one_rank_rccl(device_index: int = 0, timeout_s: int = COLLECTIVE_TIMEOUT_S) -> World:
    """A one-rank RCCL communicator whose World still exchanges through it (force_collectives):
    the multi-rank program (sampler all-gather, count and payload all-to-all-v, votes) runs
    against real RCCL on a one-GPU box (RCCL refuses two ranks on one device)."""
    global _WORLD
    dev = torch.device("cuda", device_index)
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group(backend="nccl", rank=0, world_size=1,
                                timeout=datetime.timedelta(seconds=timeout_s), device_id=dev)
        warm_collectives(dev, 1)
    _WORLD = World(rank=0, size=1, local_rank=0, device=dev, backend="nccl", force_collectives=True)
    return _WORLD


def set_world(w: World | None):
    """Install an explicit world (tests, in-process executors)."""
    global _WORLD
    _WORLD = w


def get_world() -> World:
    return _WORLD if _WORLD is not None else World()


def shutdown():
    global _WORLD
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _WORLD = None
