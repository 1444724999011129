"""Row gather (100-byte rows, random order) A/B: where the sources of one gather live.

    python tools/micro/gather_spread_ab.py [rows] [ranges]

The receive side of the multi-rank TeraSort gathers each key range (1/16 of the rank's rows)
from the block it was received into.  Measured: 16 range-confined gathers of random rows take
~84 ms where one gather over the whole table takes ~72 ms (tools/micro/ts_recv_ab.py).  This
times one range's gather (m = rows / ranges rows, random order) with its sources

* ``contiguous``: one block of m rows (the received-round layout),
* ``8 pieces``: 8 blocks of m / 8 rows spaced rows / 8 apart (a source-major receive layout),
* ``whole``: m rows drawn uniformly from the whole table.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import _lib  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402
from dryad_amd.ops._lib import ptr, stream_of  # noqa: E402


def timed(fn, reps=3):
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1)
        best = t if best is None else min(best, t)
    return best


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dev = torch.device("cuda", 0)
    rows = torch.empty((n, 100), dtype=torch.uint8, device=dev)
    out = torch.empty((n // R + 1024, 100), dtype=torch.uint8, device=dev)
    TS.generate(rows, 0, 7)
    m = n // R
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)

    def entries(src: torch.Tensor) -> torch.Tensor:
        perm = torch.randperm(src.shape[0], device=dev, generator=g)
        s = src[perm]
        pos = torch.arange(s.shape[0], device=dev, dtype=torch.int64)
        return ((pos << 32) | s).contiguous()          # distinct windows: no fix-up runs

    def gather(e: torch.Tensor):
        _lib.call("dr_gather_fixup", ptr(rows), ptr(out), ptr(e), ctypes.c_uint64(e.shape[0]), ctypes.c_uint32(100),
                  ctypes.c_uint32(0), ctypes.c_uint32(10), 32, ptr(flag), ptr(None), stream_of(rows))

    print(f"rows {n:.3g} ({n * 100 / 1e9:.0f} GB), one range = {m} rows ({m * 100 / 1e9:.2f} GB)", flush=True)
    b = 3
    cases = {
        "contiguous": torch.arange(b * m, (b + 1) * m, device=dev, dtype=torch.int64),
        "8 pieces": torch.cat([torch.arange(p * (n // 8) + b * (m // 8), p * (n // 8) + (b + 1) * (m // 8),
                                            device=dev, dtype=torch.int64) for p in range(8)]),
        "64 pieces": torch.cat([torch.arange(p * (n // 64) + b * (m // 64), p * (n // 64) + (b + 1) * (m // 64),
                                             device=dev, dtype=torch.int64) for p in range(64)]),
        "whole": torch.randint(0, n, (m,), device=dev, generator=g, dtype=torch.int64),
    }
    for name, src in cases.items():
        e = entries(src)
        t = timed(lambda: gather(e))
        print(f"gather of one range, sources {name:12s} {t:7.3f} ms  (x{R} = {t * R:6.1f} ms)", flush=True)
        del e


if __name__ == "__main__":
    main()
