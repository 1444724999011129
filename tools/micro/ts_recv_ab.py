"""Receive side of the multi-rank TeraSort (one rank of W), A/B of its round structure.

    python tools/micro/ts_recv_ab.py [W] [rows]

Runs one loopback step (bench.py --loopback-ranks W) to fill the receive buffer with exactly the
rows rank 0 would receive, then times on that buffer:

* ``rounds``: sort_received_rounds as the product runs it (per key range: E64 tile extraction with
  histograms, look-back sort, gather + fix-up), split into its kernels;
* ``rounds, win 24``: the same with 24-bit windows where a range is small enough (3 look-back
  passes instead of 4, runs of ~5 equal windows resolved by the gather's fix-up);
* ``one block``: the whole received buffer as one range (what the per-range split costs).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.models.terasort import TeraSortConfig, TeraSortLoopbackJob, KEYLEN  # noqa: E402
from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


def timed(fn, reps=2):
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
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    W = int(args[0]) if len(args) > 0 else 8
    n = int(float(args[1])) if len(args) > 1 else 1_250_000_000
    job = TeraSortLoopbackJob(TeraSortConfig(records_per_rank=n), W, 0)
    job.step()
    bufs, B = job.bufs, job.B
    M64 = (1 << 64) - 1
    # the separators and receive offsets of that step, recomputed the same way
    mine = RS.gen_samples((0, job.cfg.seed), n, 0, 0, M64, job.cfg.sample_target, 314159, job.dev)
    others = [RS.gen_samples((s * n, job.cfg.seed), n, s, s << 32, M64, job.cfg.sample_target, 314159, job.dev)
              for s in range(1, W)]
    seps = RS.separators_from_samples(torch.cat([mine] + others), W * B)
    seps_hi = [int(x) & M64 for x in seps[:, 1].tolist()]
    off = job._receive(seps)
    N = off[-1]
    print(f"W={W} B={B} received rows {N} ({N * 100 / 1e9:.1f} GB), rows per range ~{N // B}", flush=True)
    ref = TS.check(bufs.rows_in[:N])

    def rounds():
        return RS.sort_received_rounds(bufs, off, [N] * B, 0, seps_hi, B, 0, 0, KEYLEN)

    def check(tag):
        acc = TS.check(bufs.rows_out[:N])
        ok = int(acc[0]) == int(ref[0]) and int(acc[1]) == 0
        print(f"  {tag}: ok={ok} violations={int(acc[1])}", flush=True)

    t = timed(rounds)
    print(f"rounds (product)          {t:8.2f} ms", flush=True)
    check("rounds")
    # kernel split of one round structure
    e64a, e64b = bufs.ent_a.view(-1), bufs.ent_b.view(-1)
    flag = torch.zeros(2, dtype=torch.int32, device=job.dev)
    parts = {"extract": 0.0, "sort": 0.0, "gather": 0.0}
    for b in range(B):
        a, z = off[b], off[b + 1]
        hb = RS._range_hi_bounds(seps_hi, b)
        P = min(S.common_prefix_bits(*hb), 80)
        win = min(S.window_bits64(z - a), 32)
        r = bufs.rows_in[a:z]
        holder = {}
        parts["extract"] += timed(lambda: holder.update(x=S.extract_keys64_tile(r, 0, KEYLEN, P, e64a[a:z], hist=True)), 1)
        e, hist = holder["x"]
        parts["sort"] += timed(lambda: holder.update(s=S.sort_entries64(e, e64b[a:z], win, gen_hist=hist, err=flag[1:])), 1)
        parts["gather"] += timed(lambda: S.gather_fixup(r, holder["s"], bufs.rows_out[a:z], 0, KEYLEN, win, flag[:1]), 1)
    print("  per-kernel sums: " + ", ".join(f"{k} {v:.2f} ms" for k, v in parts.items()), flush=True)
    if "--split-only" in sys.argv:
        return

    old = S.RUN_TARGET64
    S.RUN_TARGET64 = 6.0
    t = timed(rounds)
    print(f"rounds, win 24            {t:8.2f} ms", flush=True)
    check("win24")
    S.RUN_TARGET64 = old

    def one_block():
        e, hist = S.extract_keys64_tile(bufs.rows_in[:N], 0, KEYLEN, 0, e64a[:N], hist=True)
        srt = S.sort_entries64(e, e64b[:N], 32, gen_hist=hist, err=flag[1:])
        S.gather_fixup(bufs.rows_in[:N], srt, bufs.rows_out[:N], 0, KEYLEN, 32, flag[:1])
    t = timed(one_block)
    print(f"one block                 {t:8.2f} ms", flush=True)
    check("one block")

    def gather_only(src, dst):
        e, hist = S.extract_keys64_tile(src[:N], 0, KEYLEN, 0, e64a[:N], hist=True)
        srt = S.sort_entries64(e, e64b[:N], 32, gen_hist=hist, err=flag[1:])
        torch.cuda.synchronize()
        return timed(lambda: S.gather_fixup(src[:N], srt, dst[:N], 0, KEYLEN, 32, flag[:1]))
    print(f"gather, received rows -> rows_out   {gather_only(bufs.rows_in, bufs.rows_out):8.2f} ms", flush=True)
    TS.generate(bufs.rows_in[:N], 0, job.cfg.seed)
    print(f"gather, generated rows -> rows_out  {gather_only(bufs.rows_in, bufs.rows_out):8.2f} ms", flush=True)
    # the per-range gathers again, over generated (uniformly random) rows in the same regions
    tg = 0.0
    for b in range(B):
        a, z = off[b], off[b + 1]
        r = bufs.rows_in[a:z]
        e, hist = S.extract_keys64_tile(r, 0, KEYLEN, 0, e64a[a:z], hist=True)
        srt = S.sort_entries64(e, e64b[a:z], 32, gen_hist=hist, err=flag[1:])
        torch.cuda.synchronize()
        tg += timed(lambda: S.gather_fixup(r, srt, bufs.rows_out[a:z], 0, KEYLEN, 32, flag[:1]), 1)
    print(f"per-range gathers, generated rows       {tg:8.2f} ms", flush=True)
    bufs.rows_out[:N].copy_(bufs.rows_in[:N])
    print(f"gather, generated rows_out -> rows_in {gather_only(bufs.rows_out, bufs.rows_in):8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
