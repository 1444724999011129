"""Stored-output write path: where the in-step write loses against the writer alone.

The stored TeraSort replaces its output table every step (ToStore(delete_if_exists=True)): the
old parts are renamed away and unlinked by a background thread (io/partfile.delete) while the new
parts are written.  This probe writes the same 8-file output (io/writer.write_device_pieces) under
each pattern, repeated so every pattern runs against a page cache that holds the previous output:

  fresh      new files, previous set already unlinked (synchronously, untimed)
  bg-unlink  new files while a thread unlinks the previous set (the bench's pattern)
  trunc      the previous set's files opened with O_TRUNC (truncation inside the timed write)
  recycle    the previous set renamed to the new names and overwritten in place (reuse=True)

    python tools/micro/writeback_probe2.py [GB] [dir]
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.io import writer as WR  # noqa: E402


def dirty() -> float:
    with open("/proc/meminfo") as f:
        for ln in f:
            if ln.startswith("Dirty:"):
                return round(int(ln.split()[1]) / 1e6, 1)
    return -1.0


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 15
    d = sys.argv[2] if len(sys.argv) > 2 else "/tmp/wbprobe2"
    os.makedirs(d, exist_ok=True)
    n = int(gb * 1e9)
    k = 8
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    bounds = [(n * j // k) for j in range(k + 1)]
    gen = [0]

    def names():
        gen[0] += 1
        return [f"{d}/g{gen[0]}_{j}" for j in range(k)]

    prev = names()
    WR.write_device_pieces(prev, x, bounds)
    os.sync()
    for rep in range(3):
        for mode in ("fresh", "bg-unlink", "trunc", "recycle"):
            new = names()
            th = None
            t_unlink = [0.0]
            if mode == "fresh":
                for p in prev:
                    os.remove(p)
            elif mode == "bg-unlink":
                moved = []
                for p in prev:
                    os.replace(p, p + ".del")
                    moved.append(p + ".del")

                def unlink():
                    t0 = time.perf_counter()
                    for q in moved:
                        os.remove(q)
                    t_unlink[0] = time.perf_counter() - t0
                th = threading.Thread(target=unlink)
                th.start()
            elif mode == "trunc":
                new = prev
            else:
                for p, q in zip(prev, new):
                    os.replace(p, q)
            d0 = dirty()
            t0 = time.perf_counter()
            WR.write_device_pieces(new, x, bounds, reuse=(mode == "recycle"))
            dt = time.perf_counter() - t0
            if th is not None:
                th.join()
            extra = f"  background unlink {t_unlink[0]:.2f} s" if th is not None else ""
            print(f"rep {rep} {mode:<10} {n / 1e9 / dt:6.1f} GB/s ({dt:.2f} s)  dirty {d0} -> {dirty()} GB{extra}",
                  flush=True)
            prev = new
    for f in os.listdir(d):
        os.remove(os.path.join(d, f))


if __name__ == "__main__":
    main()
