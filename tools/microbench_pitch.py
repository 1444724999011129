"""TeraSort in HBM with the input rows at a 100-byte vs a 128-byte pitch: generator (+ E64 keys),
compact radix sort, row gather with the run fix-up -- timed phase by phase, outputs compared.

    python tools/microbench_pitch.py [rows]

At a 128-byte pitch every random row read of the gather is exactly one aligned HBM line instead
of ~1.78 lines; the generator writes 28% more bytes.
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
                                                   ctypes.c_void_p, ctypes.c_void_p]
    lib.dr_gather_fixup_pitch128.restype = ctypes.c_int
    lib.dr_gather_fixup_pitch128.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_u64, c_u32, c_u32,
                                            c_u32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]

    def run(pitch):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        if pitch == 100:
            rows = buf[: n * 100].view(n, 100)
            TS.generate_with_keys64(rows, 0, 7, keys)
        else:
            rows = buf.view(n, 128)
            _lib.check(lib.dr_terasort_gen_keys64_pitch128(ptr(buf), c_u64(n), c_u64(0), c_u64(7), ptr(keys), c_u32(0),
                                                           None, stream_of(buf)), "gen pitch128")
        ev[1].record()
        srt = S.sort_entries64(keys, tmp, 32)
        ev[2].record()
        flag.zero_()
        if pitch == 100:
            S.gather_fixup(rows, srt, out, 0, 10, 32, flag)
        else:
            _lib.check(lib.dr_gather_fixup_pitch128(ptr(buf), ptr(out), ptr(srt), c_u64(n), c_u32(100), c_u32(0),
                                                    c_u32(10), 32, ptr(flag), stream_of(buf)), "gather pitch128")
        ev[3].record()
        torch.cuda.synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(3)], int(flag.item())

    res = {}
    for rnd in range(3):
        for pitch in (100, 128):
            (g, s, ga), bad = run(pitch)
            acc = TS.check(out)
            torch.cuda.synchronize()
            res[pitch] = acc.tolist()
            print(f"round {rnd} pitch {pitch}: gen {g:.2f} ms  sort {s:.2f} ms  gather {ga:.2f} ms  total "
                  f"{g + s + ga:.2f} ms  overflow={bad} check={res[pitch]}", flush=True)
    print("outputs identical (hash, order):", res[100] == res[128] and res[100][1] == 0, flush=True)


if __name__ == "__main__":
    main()
