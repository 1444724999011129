"""Microbenchmarks of the whole-partition aggregate kernel (reduce.hip) and the device hash join
(hashjoin.hip) against torch reductions and the sort-merge join, interleaved in one process.

    python tools/micro/microbench_ops.py [rows]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import reduce as RD  # noqa: E402
from dryad_amd.ops import relational as R  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    dev = "cuda"
    a = torch.randint(0, 1 << 40, (n,), dtype=torch.int64, device=dev)
    f = torch.rand(n, dtype=torch.float64, device=dev)
    m = (a & 7) == 0
    for name, fn, nbytes in (
            ("reduce Sum(int64)", lambda: RD.reduce_multi(n, [(RD.SUM, a, None)], dev), 8 * n),
            ("torch a.sum()", lambda: a.sum().item(), 8 * n),
            ("reduce Sum+Min+Max(f64), one pass", lambda: RD.reduce_multi(
                n, [(RD.SUM, f, None), (RD.MIN, f, None), (RD.MAX, f, None)], dev), 8 * n),
            ("torch f.sum/min/max, three passes", lambda: (f.sum().item(), f.min().item(), f.max().item()), 24 * n),
            ("reduce Count|p + Sum|p + First|p", lambda: RD.reduce_multi(
                n, [(RD.COUNT, None, m), (RD.SUM, a, m), (RD.FIRST, None, m)], dev), 9 * n)):
        dt = timed(fn)
        print(f"{name:40s} n={n:.2e}: {dt * 1e3:8.2f} ms  {nbytes / dt / 1e12:5.2f} TB/s", flush=True)
    del a, f, m
    torch.cuda.empty_cache()
    for no, ni in ((1 << 28, 1 << 16), (1 << 28, 1 << 22), (1 << 28, 1 << 26), (1 << 27, 1 << 27)):
        ko = torch.randint(0, ni, (no,), dtype=torch.int64, device=dev)
        ki = torch.randperm(ni, device=dev)
        eo, b0, lm = R.build_keys([ko])
        ei, _, _ = R.build_keys([ki])

        def sort_merge():
            so = S.sort_entries_hybrid(eo.clone(), b0)
            si = S.sort_entries_hybrid(ei.clone(), b0)
            return R.merge_join_pairs(so, si, lm)
        th = timed(lambda: R.hash_join_pairs(eo, ei, lm), 3)
        ts = timed(sort_merge, 3)
        print(f"join outer={no:.1e} inner={ni:.1e}: hash {th * 1e3:8.2f} ms   sort-merge {ts * 1e3:8.2f} ms",
              flush=True)
        del ko, ki, eo, ei
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
