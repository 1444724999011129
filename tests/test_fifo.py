"""FIFO channels and subgraph vertices (SURVEY C-5; reference channelfifo.h:27-241,
subgraphvertex.h:20-202): ordering, back pressure, end of stream, failure propagation and early
stop, over the native BlockFifo (csrc/runtime/fifo.h)."""
import itertools
import threading

import pytest

from dryad_amd import native
from dryad_amd.runtime.fifo import ABORTED, CLOSED, OK, TIMEOUT, FifoChannel, FifoError, run_subgraph

pytestmark = pytest.mark.timeout(60)


def test_native_fifo_status_codes_and_back_pressure():
    f = native.runtime().BlockFifo(8)
    assert f.put(b"abcdef", 0) == OK
    assert f.put(b"ghij", 0) == TIMEOUT          # 10 bytes > capacity 8: full
    assert f.queued_bytes() == 6
    assert f.get(0) == (OK, b"abcdef")
    assert f.put(b"0123456789abcdef", 0) == OK   # an oversized block passes an empty queue
    assert f.get(0)[0] == OK
    assert f.get(0) == (TIMEOUT, None)
    f.close()
    assert f.get(-1) == (CLOSED, None)
    assert f.put(b"x", 0) == CLOSED
    g = native.runtime().BlockFifo(64)
    g.abort("upstream vertex failed")
    assert g.get(-1) == (ABORTED, None) and g.error() == "upstream vertex failed"


def test_channel_streams_in_order_with_bounded_memory():
    ch = FifoChannel(capacity_bytes=4096, batch=100)
    n = 50_000
    t = threading.Thread(target=ch.write, args=(range(n),))
    t.start()
    got = list(ch)
    t.join()
    assert got == list(range(n))
    st = ch.stats()
    assert st["records"] == n and st["blocks"] == n // 100
    assert st["peak_bytes"] <= 4096 + 1024       # capacity plus at most one block's overshoot


def test_producer_failure_reaches_the_consumer():
    ch = FifoChannel(capacity_bytes=1 << 20, batch=10)
    seen = []

    def bad():
        yield from range(25)
        raise ValueError("disk gone")

    def prod():
        try:
            ch.write(bad())
        except ValueError as e:
            seen.append(e)

    t = threading.Thread(target=prod)
    t.start()
    with pytest.raises(FifoError, match="disk gone"):
        list(ch)
    t.join()
    assert seen


def test_subgraph_matches_sequential_pipeline():
    src = list(range(100_000))
    vs = [lambda it: (x * 3 for x in it), lambda it: (x for x in it if x % 7), lambda it: (x + 1 for x in it)]
    got = run_subgraph(src, vs, capacity_bytes=1 << 16, batch=256)
    assert got == [x * 3 + 1 for x in src if (x * 3) % 7]


def test_subgraph_early_stop_releases_producers():
    # an infinite source: the Take-like last vertex must stop the whole chain without hanging
    vs = [lambda it: (x * 2 for x in it), lambda it: itertools.islice(it, 1000)]
    got = run_subgraph(itertools.count(), vs, capacity_bytes=1 << 14, batch=64)
    assert got == [2 * x for x in range(1000)]


def test_subgraph_vertex_failure_is_raised():
    def boom(it):
        for x in it:
            if x == 5000:
                raise RuntimeError("vertex 1 failed")
            yield x

    with pytest.raises(RuntimeError, match="vertex 1 failed"):
        run_subgraph(range(10**6), [lambda it: iter(it), boom, lambda it: (x for x in it)],
                     capacity_bytes=1 << 14, batch=64)
