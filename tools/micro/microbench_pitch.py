"""TeraSort in HBM with the input rows at a 100-byte vs a 128-byte pitch: generator (+ E64 keys),
compact radix sort, row gather with the run fix-up -- timed phase by phase, outputs compared.

    python tools/micro/microbench_pitch.py [rows] [--span r1,r2,...] [--xcd]

``--span``: only the 128-byte-pitch gather, for several row counts inside one allocation (ns per
row against the span of the random reads).

At a 128-byte pitch every random row read of the gather is exactly one aligned HBM line instead
of ~1.78 lines; the generator writes 28% more bytes.
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import _lib  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402
from dryad_amd.ops._lib import c_u32, c_u64, ptr, stream_of  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    dev = torch.device("cuda", 0)
    buf = torch.empty(n * 128, dtype=torch.uint8, device=dev)
    out = torch.empty((n, 100), dtype=torch.uint8, device=dev)
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    tmp = out.view(-1)[: n * 8].view(torch.int64)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = _lib.lib()
    lib.dr_terasort_gen_keys64_pitch128.restype = ctypes.c_int
    lib.dr_terasort_gen_keys64_pitch128.argtypes = [ctypes.c_void_p, c_u64, c_u64, c_u64, ctypes.c_void_p, c_u32,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.dr_gather_fixup_pitch128.restype = ctypes.c_int
    lib.dr_gather_fixup_pitch128.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_u64, c_u32, c_u32,
                                            c_u32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]

    if "--xcd" in sys.argv:
        # gather timing with synthetic entries (window = position: no fix-up runs): sources random
        # over the whole table vs random inside 1/8 of it chosen by the output chunk's XCD
        # (workgroup b of the 16384-workgroup grid-stride gather runs on XCD b % 8, chunk c on b = c % 16384)
        rows_p = buf.view(n, 128)
        _lib.check(lib.dr_terasort_gen_keys64_pitch128(ptr(rows_p), c_u64(n), c_u64(0), c_u64(7), ptr(keys), c_u32(0),
                                                       None, None, stream_of(buf)), "gen pitch128")
        pos = out.view(-1)[: n * 8].view(torch.int64)          # scratch (the gather overwrites it)
        blk = n // 8
        for mode in ("random", "xcd-local", "random", "xcd-local"):
            g = torch.Generator(device=dev).manual_seed(5)
            torch.randint(0, 1 << 62, (n,), out=keys, generator=g, device=dev)
            if mode == "random":
                keys.remainder_(n)
            else:
                keys.remainder_(blk)
                torch.arange(n, out=pos)
                pos.div_(256, rounding_mode="floor").remainder_(8).mul_(blk)
                keys.add_(pos)
            torch.arange(n, out=pos)
            keys.bitwise_or_(pos.bitwise_left_shift_(32))
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.check(lib.dr_gather_fixup_pitch128(ptr(rows_p), ptr(out), ptr(keys), c_u64(n), c_u32(100),
                                                        c_u32(0), c_u32(10), 32, ptr(flag), ptr(None), stream_of(buf)), "gather")
                e1.record()
                torch.cuda.synchronize()
                best = e0.elapsed_time(e1) if best is None else min(best, e0.elapsed_time(e1))
            print(f"{mode:10s} sources, {n:.3g} rows ({n * 128 / 2**30:.0f} GiB): gather {best:.2f} ms", flush=True)
        return

    if "--span" in sys.argv:
        for m in [int(float(x)) for x in sys.argv[sys.argv.index("--span") + 1].split(",")]:
            if m > n:
                continue
            rows_m = buf[: m * 128].view(m, 128)
            _lib.check(lib.dr_terasort_gen_keys64_pitch128(ptr(rows_m), c_u64(m), c_u64(0), c_u64(7), ptr(keys),
                                                           c_u32(0), None, None, stream_of(buf)), "gen pitch128")
            srt = S.sort_entries64(keys[:m], tmp[:m], 32, err=S.lookback_error())
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.check(lib.dr_gather_fixup_pitch128(ptr(rows_m), ptr(out), ptr(srt), c_u64(m), c_u32(100),
                                                        c_u32(0), c_u32(10), 32, ptr(flag), ptr(None), stream_of(buf)), "gather")
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1)
                best = t if best is None else min(best, t)
            print(f"span {m * 128 / 2**30:7.1f} GiB ({m:.3g} rows): gather {best:7.2f} ms = {best * 1e6 / m:.3f} ns/row",
                  flush=True)
        return

    def run(pitch):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        if pitch == 100:
            rows = buf[: n * 100].view(n, 100)
            TS.generate_with_keys64(rows, 0, 7, keys)
        else:
            rows = buf.view(n, 128)
            _lib.check(lib.dr_terasort_gen_keys64_pitch128(ptr(buf), c_u64(n), c_u64(0), c_u64(7), ptr(keys), c_u32(0),
                                                           None, None, stream_of(buf)), "gen pitch128")
        ev[1].record()
        srt = S.sort_entries64(keys, tmp, 32, err=S.lookback_error())
        ev[2].record()
        flag.zero_()
        if pitch == 100:
            S.gather_fixup(rows, srt, out, 0, 10, 32, flag)
        else:
            _lib.check(lib.dr_gather_fixup_pitch128(ptr(buf), ptr(out), ptr(srt), c_u64(n), c_u32(100), c_u32(0),
                                                    c_u32(10), 32, ptr(flag), ptr(None), stream_of(buf)), "gather pitch128")
        ev[3].record()
        torch.cuda.synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(3)], int(flag.item())

    variants = [(100, 1), (128, 1)]
    res = {}
    for rnd in range(3):
        for pitch, stash in variants:
            (g, s, ga), bad = run(pitch)
            acc = TS.check(out)
            torch.cuda.synchronize()
            res[(pitch, stash)] = acc.tolist()
            print(f"round {rnd} pitch {pitch}: gen {g:.2f} ms  sort {s:.2f} ms  gather {ga:.2f} ms  total "
                  f"{g + s + ga:.2f} ms  overflow={bad} check={res[(pitch, stash)]}", flush=True)
    vals = list(res.values())
    print("outputs identical (hash, order):", all(v == vals[0] for v in vals) and vals[0][1] == 0, flush=True)


if __name__ == "__main__":
    main()
