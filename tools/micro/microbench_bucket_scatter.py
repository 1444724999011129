"""Microbenchmark: bucket scatter of 100-byte rows (the send-buffer pack of the distributed
TeraSort), ms and GB/s moved (rows read + written), for the kernel chosen by
DRYAD_BUCKET_SCATTER_V2 (1: 16-byte pieces + register prefetch, 0: dword loads).

    python tools/micro/microbench_bucket_scatter.py [rows=3e8] [buckets=8]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import sort as S  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 300_000_000
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rows = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    rows.view(torch.int32)[:, :1].random_()       # content does not matter; touch the pages
    e = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    e[:, 1] = torch.randint(0, nb, (n,), device="cuda")
    out = torch.empty_like(rows)
    for _ in range(2):
        S.bucket_scatter_rows(e, rows, out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        S.bucket_scatter_rows(e, rows, out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ms = sorted(ts)[2] * 1e3
    print(f"bucket_scatter_rows n={n} buckets={nb} v2={os.environ.get('DRYAD_BUCKET_SCATTER_V2', '1')}: "
          f"{ms:.2f} ms, {2 * n * 100 / ms / 1e6:.0f} GB/s")


if __name__ == "__main__":
    main()
