"""Per-rank phases of the multi-rank TeraSort program at full size on one GPU, timed one by one.

    python tools/micro/ts_rank_phases.py [rows]

* (the send side of generated inputs: tools/micro/ts_send_ab.py)
* receiver of stored-row inputs: E64 key extraction from 100-byte rows (row per lane / LDS tiles with the histograms),
  look-back radix sort, row gather + fix-up;
* ``--locality``: the row gather again with sources confined to windows of 2^k rows (how much of
  the random 100-byte row reads a locality-clustered layout would turn into cache hits).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


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
    dev = torch.device("cuda", 0)
    rows = torch.empty((n, 100), dtype=torch.uint8, device=dev)
    out = torch.empty((n, 100), dtype=torch.uint8, device=dev)
    ent = torch.empty((n, 2), dtype=torch.int64, device=dev)        # E128 (sender) / 2 x E64 (receiver)
    seed = 7
    print(f"rows {n:.3g} ({n * 100 / 1e9:.0f} GB)", flush=True)

    # ---- receiver (one range block of n rows)
    TS.generate(rows, 0, seed)
    e64a, e64b = ent.view(-1)[:n], ent.view(-1)[n: 2 * n]
    t = timed(lambda: S.extract_keys64(rows, 0, 10, 0, e64a))
    print(f"extract E64, row per lane  {t:8.2f} ms", flush=True)
    t = timed(lambda: S.extract_keys64_tile(rows, 0, 10, 0, e64a, hist=True))
    print(f"extract E64, LDS tiles+hist{t:8.2f} ms", flush=True)
    win = S.window_bits64(n)
    err = S.lookback_error()

    def srt64():
        e, h = S.extract_keys64_tile(rows, 0, 10, 0, e64a, hist=True)
        return S.sort_entries64(e, e64b, win, gen_hist=h, err=err)
    t_x = timed(lambda: S.extract_keys64_tile(rows, 0, 10, 0, e64a, hist=True))
    t = timed(srt64)
    print(f"look-back sort ({win} bits)  {t - t_x:8.2f} ms  err={int(err.item())}", flush=True)
    s = srt64()
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    t = timed(lambda: S.gather_fixup(rows, s, out, 0, 10, win, flag))
    print(f"gather + fix-up (100-byte) {t:8.2f} ms  overflow={int(flag.item())}", flush=True)
    if "--locality" not in sys.argv:
        return

    # ---- gather locality: entry i = (i << 32) | src(i), src a permutation inside windows of 2^k rows
    pos = e64b
    A = 0x9E3779B1
    for k in (None, 28, 26, 24, 22, 21, 20, 19, 18):
        chunk = 1 << 26
        for a in range(0, n, chunk):
            z = min(n, a + chunk)
            i = torch.arange(a, z, device=dev, dtype=torch.int64)
            if k is None:
                src = (i * A) % n
            else:
                m = (1 << k) - 1
                src = (i & ~m) + (((i & m) * A) & m)
                src = torch.clamp(src, max=n - 1)
            e64a[a:z] = (i << 32) | src
        t = timed(lambda: S.gather_fixup(rows, e64a, out, 0, 10, 32, flag))
        span = "whole table" if k is None else f"2^{k} rows = {(1 << k) * 100 / 2**20:.0f} MiB"
        print(f"gather, sources in {span:24s} {t:8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
