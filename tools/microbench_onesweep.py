"""A/B of the compact (E64) radix sort: per-pass count + scatter (dr_sort_u64) against the
single-histogram look-back sort (dr_sort_u64_onesweep), on the TeraSort generator's entries.

    python tools/microbench_onesweep.py [n]
"""
import ctypes
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
    base = torch.empty(n, dtype=torch.int64, device="cuda")
    rows = torch.empty((min(n, 1 << 26), 100), dtype=torch.uint8, device="cuda")
    # entries of n records: generate in chunks through a small row buffer
    c = rows.shape[0]
    for a in range(0, n, c):
        m = min(c, n - a)
        TS.generate_with_keys64(rows[:m], a, 7, base[a:a + m])
    del rows
    ent = torch.empty_like(base)
    tmp = torch.empty_like(base)
    flag = ctypes.c_int(0)
    ws_old = S._workspace(n, base.device)
    ws_os = S._onesweep_workspace(n, base.device)

    def old():
        _lib.call("dr_sort_u64", S.ptr(ent), S.ptr(tmp), S.c_u64(n), 32, 64, S.ptr(ws_old), S.stream_of(ent),
                  ctypes.byref(flag))

    lib = _lib.lib()
    lib.dr_sort64_onesweep_set_items.argtypes = [ctypes.c_int]
    lib.dr_sort64_onesweep_set_items.restype = None

    def new_items(items):
        lib.dr_sort64_onesweep_set_items(items)
        _lib.call("dr_sort_u64_onesweep", S.ptr(ent), S.ptr(tmp), S.c_u64(n), 32, 64, S.ptr(ws_os),
                  S.c_u64(ws_os.numel()), None, S.c_u32(0), S.stream_of(ent), ctypes.byref(flag))
        lib.dr_sort64_onesweep_set_items(32)

    results = {}
    for rnd in range(2):
        for name, fn in (("count+scatter", old), ("onesweep-items32", lambda: new_items(32)),
                         ("onesweep-items16", lambda: new_items(16))):
            def run():
                ent.copy_(base)
                fn()
            med, best = timeit(run)
            cmed, _ = timeit(lambda: ent.copy_(base))
            run()
            torch.cuda.synchronize()
            res = (tmp if flag.value else ent).clone()
            results.setdefault(name, res)
            print(f"round {rnd} {name}: sort64 4 passes {med - cmed:.2f} ms (median {med:.2f}, best {best:.2f}, "
                  f"copy {cmed:.2f})", flush=True)
            del res
    S.onesweep_check(base.device)
    same = all(torch.equal(results["count+scatter"], results[f"onesweep-{i}"]) for i in ("items32", "items16"))
    w = (results["onesweep-items32"] >> 32) & 0xFFFFFFFF
    ordered = bool((w[1:] >= w[:-1]).all())
    print(f"n={n} identical={same} ordered={ordered}", flush=True)


if __name__ == "__main__":
    main()
