"""Job handles and status (reference LinqToDryad/DryadLinqQueryRuntime.cs:34-110,
IDryadLinqJobSubmission.cs:30-68)."""
from __future__ import annotations

import enum
import threading
import time

from .errors import DryadLinqJobException, ErrorCode


class JobStatus(enum.Enum):
    NotSubmitted = 0
    Waiting = 1
    Running = 2
    Success = 3
    Failure = 4
    Cancelled = 5


class JobHandle:
    """One submitted job (the IDryadLinqJobSubmission side)."""

    def __init__(self, job_id: str):
        self.job_id = job_id
        self.status = JobStatus.Waiting
        self.error: BaseException | None = None
        self.result = None
        self.events = []
        self._done = threading.Event()
        self._cancel = threading.Event()
        self.thread: threading.Thread | None = None
        self.submit_time = time.time()
        self.end_time = None

    def set_running(self):
        self.status = JobStatus.Running

    def finish(self, ok: bool, error: BaseException | None = None, result=None):
        self.status = JobStatus.Success if ok else (JobStatus.Cancelled if self._cancel.is_set() else JobStatus.Failure)
        self.error = error
        self.result = result
        self.end_time = time.time()
        self._done.set()

    def wait(self, timeout=None) -> bool:
        return self._done.wait(timeout)

    def cancel(self):
        self._cancel.set()
        pump = getattr(self, "pump", None)          # wake the job manager blocked in its pump
        if pump is not None:
            pump.post(MSG_CANCEL, 0)

    @property
    def cancelled(self) -> bool:
        return self._cancel.is_set()


MSG_RESULT, MSG_DUPLICATES, MSG_CANCEL = 1, 2, 3     # job manager pump message kinds


class DryadLinqJobInfo:
    """Result of ``Submit``: ``JobIds``, ``Wait()`` (raises on failure), ``CancelJob()``."""

    def __init__(self, handles: list[JobHandle]):
        self._handles = list(handles)

    @property
    def JobIds(self) -> list[str]:
        return [h.job_id for h in self._handles]

    @property
    def status(self) -> JobStatus:
        st = [h.status for h in self._handles]
        for s in (JobStatus.Failure, JobStatus.Cancelled, JobStatus.Running, JobStatus.Waiting):
            if s in st:
                return s
        return JobStatus.Success if st else JobStatus.NotSubmitted

    def Wait(self, timeout: float | None = None):
        for h in self._handles:
            if not h.wait(timeout):
                raise DryadLinqJobException(ErrorCode.JobStatusQueryError, f"timed out waiting for job {h.job_id}")
            if h.status != JobStatus.Success:
                raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed, f"job {h.job_id} {h.status.name}: {h.error}", inner=h.error)
        return self

    def CancelJob(self):
        for h in self._handles:
            h.cancel()

    @property
    def events(self):
        return [e for h in self._handles for e in h.events]

    # python aliases
    wait = Wait
    cancel_job = CancelJob
