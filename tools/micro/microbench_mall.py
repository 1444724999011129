"""Does a bucket-partitioned source make the TeraSort row gather Infinity-Cache friendly?

Times the same in-HBM sort (RS.local_sort_rows: compact radix sort + fused gather) on rows in
generator order and on the same rows stably partitioned by their top key byte (256 buckets), so the
gather of each output range reads one bucket.  python tools/micro/microbench_mall.py [rows]"""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


def timeit(fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 500_000_000
    buckets = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dev = torch.device("cuda")
    rows = torch.empty((n, 100), dtype=torch.uint8, device=dev)
    TS.generate(rows, 0, 7)
    out = torch.empty_like(rows)
    ea = torch.empty((n + 1024, 2), dtype=torch.int64, device=dev)
    eb = torch.empty_like(ea)
    t_a = timeit(lambda: RS.local_sort_rows(rows, out, ea, eb, 0, 10))
    ref = out[:1000].clone()
    # stable partition of the rows by key range (equal-width ranges of the first key bytes)
    e = S.extract_keys(rows, 0, 10, 0, out=ea[:n])
    seps = torch.zeros((buckets - 1, 2), dtype=torch.int64, device=dev)
    for j in range(1, buckets):
        v = (j << 64) // buckets
        seps[j - 1, 1] = v - (1 << 64) if v >= (1 << 63) else v
    S.range_dest(e, seps, 0)
    S.bucket_scatter_rows(e, rows, out)
    rows.copy_(out)
    t_b = timeit(lambda: RS.local_sort_rows(rows, out, ea, eb, 0, 10))
    assert torch.equal(out[:1000], ref)
    gb = n * 100 / 1e9
    print(f"n={n} ({gb:.0f} GB) buckets={buckets}: generator order {t_a * 1e3:.1f} ms, "
          f"bucket-partitioned {t_b * 1e3:.1f} ms ({gb / t_a:.0f} -> {gb / t_b:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
