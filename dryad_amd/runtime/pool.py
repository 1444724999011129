"""Vertex-host pools: the ProcessService / LocalScheduler layer of the CPU executor.

Reference: ProcessService (per-worker daemon launching VertexHost processes, ProcessService.cs:
42-752), LocalScheduler (slot matching, LocalScheduler.cs:132-268) and LocalJobSubmission (N worker
processes on localhost, LocalJobSubmission.cs:97-147).  ``ProcessPool`` keeps one long-lived vertex
host process per slot (fault containment: a crashing vertex kills only its host, which is
restarted); ``ThreadPool`` runs vertices in threads of the client process (fast path for tests and
LocalDebug-adjacent use).  Both expose acquire / send / poll / release / kill.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import queue
import threading
from multiprocessing.connection import wait as mp_wait

from ..native import runtime as native_runtime


class ProcessPool:
    """One vertex-host *program* per slot (python -m dryad_amd.runtime.vertexhost), connected back
    over an AF_UNIX socket; a host that dies is detected by EOF on its connection and restarted."""

    def __init__(self, n: int, locality_delay: float = 0.0):
        import secrets
        import subprocess
        import tempfile
        from multiprocessing.connection import Listener
        self._subprocess = subprocess
        self.n = max(1, int(n))
        self._dir = tempfile.mkdtemp(prefix="dryad-vh-")
        self._addr = os.path.join(self._dir, "jm.sock")
        self._key = secrets.token_bytes(16)
        self._listener = Listener(self._addr, family="AF_UNIX", authkey=self._key)
        self._procs = [None] * self.n
        self._conns = [None] * self.n
        self._current = [None] * self.n           # (vertex, version) running on the slot
        self.sched = native_runtime().Scheduler(self.n, locality_delay)
        for i in range(self.n):
            self._launch(i)
        for i in range(self.n):
            self._accept(i)
        self._pump = None
        self._watcher = None
        self._armed = threading.Event()
        self._wake_r, self._wake_w = mp.Pipe(duplex=False)
        self._closed = False

    # ---- event-driven results: a watcher thread posts a pump message when a host has something
    # to say; the job manager then collects it with poll(0) on its own thread and re-arms
    def attach(self, pump, kind: int):
        self._pump, self._kind = pump, kind
        if self._watcher is None:
            self._watcher = threading.Thread(target=self._watch, daemon=True, name="dryad-vh-watch")
            self._watcher.start()
        self._armed.set()

    def rearm(self):
        self._armed.set()

    def _conns_changed(self):
        if self._watcher is not None:
            try:
                self._wake_w.send_bytes(b"x")
            except OSError:
                pass

    def _watch(self):
        while not self._closed:
            self._armed.wait()
            if self._closed:
                return
            conns = [c for c in list(self._conns) if c is not None]
            try:
                ready = mp_wait(conns + [self._wake_r])
            except (OSError, ValueError):            # a connection closed under us: let poll() see
                ready = conns
            if self._wake_r in ready:
                try:
                    while self._wake_r.poll():
                        self._wake_r.recv_bytes()
                except (OSError, EOFError):
                    return
                ready = [r for r in ready if r is not self._wake_r]
                if not ready:
                    continue                         # refresh the connection list
            if self._closed:
                return
            self._armed.clear()
            pump = self._pump
            if pump is not None:
                pump.post(self._kind, 0)

    def _launch(self, i):
        import sys
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ)
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        self._procs[i] = self._subprocess.Popen(
            [sys.executable, "-m", "dryad_amd.runtime.vertexhost", "--address", self._addr, "--slot", str(i),
             "--authkey", self._key.hex()], env=env)

    def _accept(self, i):
        conn = self._listener.accept()
        conn.send(("slot?", i))
        self._conns[i] = conn
        self.sched.set_alive(i, True)

    def acquire(self, preferred=(), waited: float = 1e9):
        w = self.sched.place(list(preferred), waited)
        if w < 0:
            return None
        self.sched.set_busy(w)
        return w

    def send(self, slot, cmd):
        self._current[slot] = (cmd["vertex"], cmd["version"])
        try:
            self._conns[slot].send(cmd)
        except (BrokenPipeError, OSError):
            pass   # detected as a lost host by poll()

    def release(self, slot):
        self._current[slot] = None
        self.sched.release(slot)

    def poll(self, timeout):
        out = []
        conns = {c: i for i, c in enumerate(self._conns) if c is not None}
        live = {c for c, i in conns.items() if self._current[i] is not None}
        if not live:
            timeout = 0                              # only idle hosts to look at
        for r in mp_wait(list(conns), timeout):
            i = conns[r]
            if r not in live:                        # an idle host: died (EOF) -> restarted
                try:
                    r.recv()
                except (EOFError, OSError):
                    self._restart(i)
                continue
            try:
                res = r.recv()
            except (EOFError, OSError):
                res = self._lost(i)
            out.append((i, res))
        return out

    def _lost(self, i):
        v, ver = self._current[i]
        code = self._procs[i].poll()
        self._restart(i)
        return dict(vertex=v, version=ver, ok=False, lost=True, bad_edge=-1,
                    error=f"vertex host process {i} died (exit code {code})", bytes_read=0, bytes_written=0)

    def _restart(self, i):
        try:
            self._conns[i].close()
        except OSError:
            pass
        p = self._procs[i]
        if p is not None and p.poll() is None:
            p.kill()
            p.wait(5)
        self._launch(i)
        self._accept(i)
        self._conns_changed()

    def kill(self, slot):
        """Cancel the vertex running on a slot by killing its host (restarted immediately)."""
        self._current[slot] = None
        self._restart(slot)
        self.sched.release(slot)

    def close(self):
        self._closed = True
        self._armed.set()
        self._conns_changed()
        for c in self._conns:
            try:
                c.send(None)
            except Exception:
                pass
        for p in self._procs:
            if p is not None:
                try:
                    p.wait(3)
                except Exception:
                    p.kill()
        try:
            self._listener.close()
        except Exception:
            pass
        import shutil
        shutil.rmtree(self._dir, ignore_errors=True)

    def __del__(self):
        try:
            for p in self._procs:
                if p is not None and p.poll() is None:
                    p.kill()
        except Exception:
            pass


class ThreadPool:
    """In-process vertex execution on worker threads."""

    def __init__(self, n: int, plan_getter=None):
        self.n = max(1, int(n))
        self.sched = native_runtime().Scheduler(self.n, 0.0)
        self._q = queue.Queue()
        self._inbox = [queue.Queue() for _ in range(self.n)]
        self._current = [None] * self.n
        self._cancelled = set()
        self._plans = {}
        self._threads = []
        self._pump = None
        for i in range(self.n):
            t = threading.Thread(target=self._loop, args=(i,), daemon=True, name=f"dryad-vertex-{i}")
            t.start()
            self._threads.append(t)

    def register_plan(self, job_dir, plan):
        self._plans[job_dir] = plan

    def _loop(self, i):
        from .worker import execute_vertex
        while True:
            cmd = self._inbox[i].get()
            if cmd is None:
                return
            res = execute_vertex(cmd, self._plans.get(cmd["job"]))
            self._q.put((i, res))
            pump = self._pump
            if pump is not None:
                pump.post(self._kind, 0)

    def attach(self, pump, kind: int):
        self._pump, self._kind = pump, kind

    def rearm(self):
        pass

    def acquire(self, preferred=(), waited=1e9):
        w = self.sched.place(list(preferred), waited)
        if w < 0:
            return None
        self.sched.set_busy(w)
        return w

    def send(self, slot, cmd):
        self._current[slot] = (cmd["vertex"], cmd["version"])
        self._inbox[slot].put(cmd)

    def release(self, slot):
        self._current[slot] = None
        self.sched.release(slot)

    def poll(self, timeout):
        out = []
        try:
            item = self._q.get(timeout=timeout) if timeout else self._q.get_nowait()
        except queue.Empty:
            return out
        out.append(item)
        while True:
            try:
                out.append(self._q.get_nowait())
            except queue.Empty:
                break
        # drop results of vertices cancelled meanwhile
        return [(i, r) for i, r in out if (r["vertex"], r["version"]) not in self._cancelled]

    def kill(self, slot):
        # threads cannot be killed: mark the attempt cancelled and let it finish in the background
        if self._current[slot] is not None:
            self._cancelled.add(self._current[slot])
        self._current[slot] = None
        # the slot stays busy until the thread finishes; replace it with a fresh thread slot
        self._inbox.append(queue.Queue())
        self._current.append(None)
        new = self.sched.add_worker()
        t = threading.Thread(target=self._loop, args=(new,), daemon=True)
        t.start()
        self._threads.append(t)
        self.sched.set_alive(slot, False)

    def close(self):
        for q in self._inbox:
            q.put(None)
