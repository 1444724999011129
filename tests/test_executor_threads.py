"""Job threads of the GPU executor are bound to the rank's GPU.

The HIP current device is per host thread and a new thread starts on device 0.  A job runs on a
thread of its own (``_BaseExecutor.submit``), so without the binding every rank's launches on the
default stream (and the kernel library's device queries) would go to GPU 0 -- invisible on a
one-GPU box, fatal at 8 GPUs.  CPU test: torch.cuda.set_device is recorded, not called."""
import threading

import torch

from dryad_amd.jobinfo import JobHandle, JobStatus
from dryad_amd.parallel.comm import World
from dryad_amd.runtime import gpu_executor as GE


def _executor(device):
    ex = object.__new__(GE.GpuExecutor)
    ex.world = World(3, 8, 3, device, None)
    return ex


def test_job_thread_binds_rank_device(monkeypatch):
    calls = []
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: calls.append((threading.current_thread().name, d)))
    ex = _executor(torch.device("cuda", 3))
    seen = {}

    def run_job(outs, handle):
        seen["thread"] = threading.current_thread().name
        return {"events": []}

    ex.run_job = run_job
    h = JobHandle("j1")
    ex.submit([], h)
    assert h.wait(10)
    assert h.status == JobStatus.Success, h.error
    assert seen["thread"].startswith("dryad-job-")
    assert calls and calls[0][0] == seen["thread"] and calls[0][1] == torch.device("cuda", 3)


def test_cpu_world_does_not_touch_devices(monkeypatch):
    calls = []
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: calls.append(d))
    ex = _executor(torch.device("cpu"))
    ex._enter_job_thread()
    assert calls == []


def test_failed_thread_setup_fails_the_job(monkeypatch):
    def boom(d):
        raise RuntimeError("no such device")
    monkeypatch.setattr(torch.cuda, "set_device", boom)
    ex = _executor(torch.device("cuda", 5))
    ex.run_job = lambda outs, handle: {"events": []}
    h = JobHandle("j2")
    ex.submit([], h)
    assert h.wait(10)
    assert h.status == JobStatus.Failure and "no such device" in str(h.error)
