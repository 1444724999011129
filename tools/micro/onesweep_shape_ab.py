"""A/B of the look-back scatter (argv[2] = "count": of the count + scatter dr_sort_u64 passes)'s workgroup shape (csrc/kernels/sort.hip, -DDR_OS_SHAPE variant
libraries via DRYAD_KERNEL_LIB).  1.25e9 E64 entries = random 31-bit window << 33 | index, three
8-bit passes over the top 24 bits (the 1-GPU TeraSort's entry sort).  Checks: window bits
non-decreasing, stable (indices increase inside equal windows), a permutation of the input indices."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from dryad_amd.ops import sort as S  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
lookback = not (len(sys.argv) > 2 and sys.argv[2] == "count")   # "count": the count + scatter passes
g = torch.Generator(device="cuda").manual_seed(1)
src = (torch.randint(0, 1 << 31, (n,), device="cuda", generator=g, dtype=torch.int64) << 33) | torch.arange(
    n, device="cuda", dtype=torch.int64)
e = torch.empty_like(src)
tmp = torch.empty_like(src)
times = []
for _ in range(6):
    e.copy_(src)
    err = S.lookback_error()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = S.sort_entries64(e, tmp, 24, err=err, lookback=lookback)
    torch.cuda.synchronize()
    times.append((time.perf_counter() - t0) * 1e3)
    assert int(err.item()) == 0
win = (out >> 40) & ((1 << 24) - 1)
idx = out & ((1 << 33) - 1)
assert bool((win[1:] >= win[:-1]).all()), "window order"
same = win[1:] == win[:-1]
assert bool((idx[1:][same] > idx[:-1][same]).all()), "stability"
assert torch.equal(torch.sort(idx).values, torch.arange(n, device="cuda")), "permutation"
print(f"{'look-back' if lookback else 'count + scatter'}: 3 passes + hist {min(times):.2f} ms (all {[round(t, 2) for t in times]}) VALID", flush=True)
