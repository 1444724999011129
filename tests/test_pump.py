"""The job manager's event pump (csrc/runtime/pump.h, SURVEY G-10; reference DrMessagePump,
GraphManager/kernel/DrMessagePump.h:20-295): timers by deadline, cross-thread wake-ups with the
GIL released, close; and the job manager driven by it (results, duplicate timer, user cancel)."""
import threading
import time

import dryad_amd as D
from dryad_amd.native import runtime


def test_pump_orders_timers_and_posts():
    p = runtime().MessagePump()
    p.post_after(60, 2, 20)
    p.post_after(30, 2, 10)
    p.post(1, 1)
    assert p.wait(-1) == [(1, 1)]
    t = time.time()
    assert p.wait(-1) == [(2, 10)]
    assert p.wait(-1) == [(2, 20)]
    assert 0.05 <= time.time() - t < 1.0
    assert p.wait(0) == [] and p.wait(20) == []
    assert p.posted() == 3 and p.delivered() == 3


def test_pump_wakes_across_threads_and_closes():
    p = runtime().MessagePump()
    got = []

    def waiter():
        got.append(p.wait(-1))      # blocks with the GIL released
        got.append(p.wait(-1))      # woken by close() with nothing

    th = threading.Thread(target=waiter)
    th.start()
    time.sleep(0.05)
    x = sum(range(100000))          # the main thread runs while the waiter blocks
    p.post(7, x)
    time.sleep(0.05)
    p.close()
    th.join(2)
    assert not th.is_alive()
    assert got == [[(7, x)], []]
    p.post(1, 1)                    # ignored after close
    assert p.pending() == 0


def _ctx(pool, **props):
    c = D.DryadLinqContext(3)
    c._props["PoolKind"] = pool
    c._props.update(props)
    return c


def test_job_manager_runs_on_the_pump():
    for pool in ("thread", "process"):
        c = _ctx(pool)
        assert sorted(c.FromEnumerable(range(60)).Select(lambda x: x * 3)) == [x * 3 for x in range(60)]
        c.Dispose()


def test_cancel_wakes_a_blocked_job_manager():
    c = _ctx("process", FaultInjection=[dict(stage=None, partition=0, version=0, kind="slow:20")])
    info = c.FromEnumerable(range(30)).Select(lambda x: x).ToStore("mem://pump_cancel", delete_if_exists=True).Submit()
    time.sleep(1.0)
    t = time.time()
    info.CancelJob()
    try:
        info.Wait()
    except Exception:
        pass
    assert time.time() - t < 5.0        # not the 20 s straggler: the cancel message woke the manager
    c.Dispose()
