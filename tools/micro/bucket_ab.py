"""A/B of the one-rank pitch-128 sort at 1.25e9 TeraSort rows: four look-back passes on the 32-bit
window + the staged fix-up gather (bucket=0) vs three passes on 24 bits + the bucket gather
(bucket=1).  Each step regenerates the rows + entries (as the bench's read stage), then sorts.

    python tools/micro/bucket_ab.py [n]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
    dev = torch.device("cuda")
    out = torch.empty((n + 1024, 100), dtype=torch.uint8, device=dev)
    rows = torch.empty((n + 1024, 128), dtype=torch.uint8, device=dev)
    keys = torch.empty(n + 1024, dtype=torch.int64, device=dev)
    rng = torch.tensor([-1, 0], dtype=torch.int64, device=dev)
    ref = None
    orig = S.bucket_sort_ok
    for variant in ("bucket=0", "bucket=1", "bucket=0", "bucket=1"):
        on = variant.endswith("1")
        S.bucket_sort_ok = (lambda n_, k_: orig(n_, k_)) if on else (lambda n_, k_: False)
        fmt = "e64@out" if on else "e64"
        ts_gen, ts_sort = [], []
        for _ in range(4):
            home = out.view(-1)[: n * 8].view(torch.int64) if on else keys
            a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            TS.generate_with_keys64_pitch128(rows[:n], 0, 1234, home, rng, hist=True)
            b.record()
            info = {}
            got = S.sort_rows_pitch128(rows[:n], out, keys, 0, 10, keys_ready=True, stats=info, keys_fmt=fmt)
            c.record()
            torch.cuda.synchronize()
            ts_gen.append(a.elapsed_time(b))
            ts_sort.append(b.elapsed_time(c))
        acc = TS.check(got)
        print(f"{variant}: gen {sorted(ts_gen)[1]:.2f} ms, sort {sorted(ts_sort)[1]:.2f} ms (all {[round(x, 2) for x in ts_sort]}), "
              f"violations {int(acc[1])}, hash {int(acc[0])}, path: {info.get('path')}", flush=True)
        if ref is None:
            ref = int(acc[0])
        assert int(acc[1]) == 0 and int(acc[0]) == ref
    S.bucket_sort_ok = orig


if __name__ == "__main__":
    main()
