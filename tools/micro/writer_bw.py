"""HBM -> part files through io/writer.py: one file (write_device) vs k files at once
(write_device_pieces), and the device -> pinned copy rate alone.

    python tools/micro/writer_bw.py [GB] [dir]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.io import writer as WR  # noqa: E402
from dryad_amd.ops import _lib  # noqa: E402


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 20
    d = sys.argv[2] if len(sys.argv) > 2 else "/tmp/wbw"
    os.makedirs(d, exist_ok=True)
    n = int(gb * 1e9)
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    ring = WR._ring()
    cs = torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in range(0, n, WR.CHUNK):
        m = min(WR.CHUNK, n - a)
        _lib.memcpy_async(ring[(a // WR.CHUNK) % len(ring)].tensor[:m], x[a:a + m], cs)
    cs.synchronize()
    dt = time.perf_counter() - t0
    print(f"device -> pinned ring copies       {n / 1e9 / dt:7.1f} GB/s", flush=True)
    for k in (1, 2, 4, 8):
        paths = [f"{d}/f{j}" for j in range(k)]
        t0 = time.perf_counter()
        if k == 1:
            WR.write_device(paths[0], x)
        else:
            bounds = [(n * j // k) for j in range(k + 1)]
            WR.write_device_pieces(paths, x, bounds)
        dt = time.perf_counter() - t0
        print(f"write {gb:.0f} GB into {k} file(s)        {n / 1e9 / dt:7.1f} GB/s", flush=True)
        for p in paths:
            os.remove(p)


if __name__ == "__main__":
    main()
