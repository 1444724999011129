"""Interleaved A/B microbenchmark of sort/gather kernel variants in one process (guide §5.4 rule 24).

    python tools/microbench_sort.py [n]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


def timeit(fn, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2] * 1e3, ts[0] * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
    bufs = RS.SortBuffers.allocate(n, 100, "cuda")
    TS.generate(bufs.rows_in[:n], 0, 7)
    rows = bufs.rows_in[:n]
    e = S.extract_keys(rows, 0, 10, 0, out=bufs.ent_a[:n])
    base = e.clone()
    res = {}
    for rnd in range(2):
        for items, v2 in ((8, False), (16, True)):
            S.set_sort_items(items)
            S.set_scatter_v2(v2)

            def full():
                bufs.ent_a[:n].copy_(base)
                S.sort_entries(bufs.ent_a[:n], 48, 128, tmp=bufs.ent_b[:n])

            def pref():
                bufs.ent_a[:n].copy_(base)
                S.sort_entries_prefix(bufs.ent_a[:n], 48, tmp=bufs.ent_b[:n])

            st = {}

            def hyb():
                bufs.ent_a[:n].copy_(base)
                S.sort_entries_hybrid(bufs.ent_a[:n], 48, 128, tmp=bufs.ent_b[:n], stats=st)

            def hyb_b():
                bufs.ent_a[:n].copy_(base)
                S.sort_entries_hybrid(bufs.ent_a[:n], 48, 128, tmp=bufs.ent_b[:n], hi_bounds=(0, 2**64 - 1))

            res.setdefault(f"sort10 items={items} v2={v2}", []).append(timeit(full))
            res.setdefault(f"sort8+fixup items={items} v2={v2}", []).append(timeit(pref))
            res.setdefault(f"hybrid items={items} v2={v2}", []).append(timeit(hyb))
            res.setdefault(f"hybrid(bounds) items={items} v2={v2}", []).append(timeit(hyb_b))
            print("hybrid path:", st, flush=True)
        srt3 = S.sort_entries(bufs.ent_a[:n].copy_(base), 104, 128, tmp=bufs.ent_b[:n]).clone()
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        res.setdefault("seg_sort_runs only", []).append(timeit(lambda: S._lib.call(
            "dr_seg_sort_runs", S.ptr(srt3), S.c_u64(n), 40, S.c_u64(2**64 - 1), S.c_u64(2**64 - 1),
            S.ptr(flag), S.stream_of(srt3))))
        res.setdefault("hi_range only", []).append(timeit(lambda: S.hi_range(base)))
        S.set_sort_items(8)
        # reference: rocPRIM radix sort through torch.sort (int64 keys + int64 indices, stable)
        keys = base[:, 1].clone()
        res.setdefault("torch.sort int64 stable (rocPRIM ref)", []).append(
            timeit(lambda: torch.sort(keys, stable=True)))
        srt = S.sort_entries(bufs.ent_a[:n].copy_(base), 48, 128, tmp=bufs.ent_b[:n])
        for v4 in (False, True):
            S.set_gather_v4(v4)
            res.setdefault(f"gather v4={v4}", []).append(
                timeit(lambda: S.gather_rows(rows, entries=srt, out=bufs.rows_out[:n])))
        res.setdefault("copy entries (ref)", []).append(timeit(lambda: bufs.ent_b[:n].copy_(base)))
        res.setdefault("extract", []).append(timeit(lambda: S.extract_keys(rows, 0, 10, 0, out=bufs.ent_a[:n])))
    gb = n * 16 / 1e9
    for k, v in res.items():
        med = min(x[0] for x in v)
        print(f"{k:28s} median_ms={med:8.2f}  (entries {gb:.1f} GB)  all={[round(x[0], 2) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
