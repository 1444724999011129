"""Interleaved A/B microbenchmark of the compact (E64) sort: scatter tile size and the gather.

    python tools/microbench_sort64.py [n]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dryad_amd.ops import _lib  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000_000
    rows = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    ent = torch.empty(n, dtype=torch.int64, device="cuda")
    tmp = torch.empty(n, dtype=torch.int64, device="cuda")
    base = torch.empty(n, dtype=torch.int64, device="cuda")
    TS.generate_with_keys64(rows, 0, 7, base)
    lib = _lib.lib()
    lib.dr_sort64_set_items.argtypes = [_lib.c_i32]
    lib.dr_sort64_set_items.restype = None
    lib.dr_sort64_set_variant.argtypes = [_lib.c_i32]
    lib.dr_sort64_set_variant.restype = None
    ref = None
    for rnd in range(2):
        for items, var in ((16, 3), (16, 4)):
            lib.dr_sort64_set_items(items)
            lib.dr_sort64_set_variant(var)

            def srt():
                ent.copy_(base)
                S.sort_entries64(ent, tmp, 32)

            def cp():
                ent.copy_(base)
            med, best = timeit(srt)
            cmed, _ = timeit(cp)
            srt()
            torch.cuda.synchronize()
            res = ent.clone()
            if ref is None:
                ref = res
            same = bool(torch.equal(res, ref))
            print(f"round {rnd} items={items} variant={var}: sort64 4 passes {med - cmed:.2f} ms (median {med:.2f}, "
                  f"copy {cmed:.2f}) same_as_first={same}", flush=True)
    lib.dr_sort64_set_items(16)
    lib.dr_sort64_set_variant(3)
    # gather: plain vs nontemporal output stores
    lib.dr_gather_fixup_set_nt.argtypes = [_lib.c_i32]
    lib.dr_gather_fixup_set_nt.restype = None
    ent.copy_(base)
    srt_e = S.sort_entries64(ent, tmp, 32)
    out = torch.empty_like(rows)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    for rnd in range(2):
        for nt in (0, 1):
            lib.dr_gather_fixup_set_nt(nt)
            med, best = timeit(lambda: S.gather_fixup(rows, srt_e, out, 0, 10, 32, flag))
            print(f"round {rnd} gather nt={nt}: {med:.2f} ms (best {best:.2f})", flush=True)
    lib.dr_gather_fixup_set_nt(0)


if __name__ == "__main__":
    main()
