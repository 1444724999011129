"""Does an MSD-first radix sort pay on MI355X?  One 8-bit MSD partition pass over HBM, then the
remaining LSD passes bucket by bucket while each bucket (n/256 entries, ~80 MB in + out at
1.25e9 entries) stays resident in the 256 MB Infinity Cache — against the plain 4-pass LSD of the
same 32-bit window.  Interleaved in one process, results checked equal.

    python tools/micro/microbench_msd.py [entries]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import _lib  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops._lib import c_u64, ptr, stream_of  # noqa: E402


def lsd(e, tmp, ws, b, t):
    flag = ctypes.c_int(0)
    _lib.call("dr_sort_u128", ptr(e), ptr(tmp), c_u64(e.shape[0]), b, t, ptr(ws), stream_of(e), ctypes.byref(flag))
    return flag.value


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
    dev = "cuda"
    src = torch.empty((n, 2), dtype=torch.int64, device=dev)
    src[:, 1].random_()
    src[:, 0] = torch.arange(n, device=dev)
    a = torch.empty_like(src)
    b = torch.empty_like(src)
    ws = S._workspace(n, dev)
    top, win = 128, 32

    def plain():
        a.copy_(src)
        f = lsd(a, b, ws, top - win, top)
        return b if f else a

    def msd():
        a.copy_(src)
        out, starts = S.partition_pass(a, top - 8, b)
        st = starts.cpu().tolist()
        flips = None
        for k in range(256):
            lo, hi = st[k], st[k + 1]
            if hi - lo < 2:
                continue
            f = lsd(out[lo:hi], a[lo:hi], ws, top - win, top - 8)
            assert flips is None or f == flips
            flips = f
        if flips:
            # single-entry buckets stayed in `out`: move them (rare at this size)
            for k in range(256):
                if st[k + 1] - st[k] == 1:
                    a[st[k]:st[k + 1]] = out[st[k]:st[k + 1]]
            return a
        return out

    for name, fn in (("lsd 4 passes", plain), ("msd + 3 cached passes", msd)):
        fn()
        torch.cuda.synchronize()
    ts = {"lsd 4 passes": [], "msd + 3 cached passes": []}
    for _ in range(4):
        for name, fn in (("lsd 4 passes", plain), ("msd + 3 cached passes", msd)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            ts[name].append(time.perf_counter() - t0)
            if name.startswith("lsd"):
                ref = r[:, 1].clone()
            else:
                assert torch.equal(ref, r[:, 1]), "msd result differs"
    cp = src.numel() * 8 * 2 / 5.5e12   # the copy_ in each variant, subtracted
    for name, v in ts.items():
        m = sorted(v)[len(v) // 2]
        print(f"{name:26s} n={n:.2e}: {(m - cp) * 1e3:8.2f} ms (copy excluded)", flush=True)


if __name__ == "__main__":
    main()
