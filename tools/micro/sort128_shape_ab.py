"""A/B of the E128 count-matrix sort pass (csrc/kernels/sort.hip: rs_scatter_v2 at 256 threads vs
rs_scatter_w, -DDR_SORT_NT / -DDR_SORT_ITEMS variant libraries via DRYAD_KERNEL_LIB).  5e8 entries
{lo = index, hi = random}, four 8-bit passes over hi bits [0, 32).  Checks: sorted on those bits,
stable (indices increase inside equal keys), a permutation of the indices."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from dryad_amd.ops import sort as S  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 500_000_000
g = torch.Generator(device="cuda").manual_seed(3)
src = torch.empty((n, 2), dtype=torch.int64, device="cuda")
src[:, 0] = torch.arange(n, device="cuda", dtype=torch.int64)
src[:, 1] = torch.randint(0, 1 << 62, (n,), device="cuda", generator=g, dtype=torch.int64)
e = torch.empty_like(src)
tmp = torch.empty_like(src)
times = []
for _ in range(6):
    e.copy_(src)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = S.sort_entries(e, 64, 96, tmp)
    torch.cuda.synchronize()
    times.append((time.perf_counter() - t0) * 1e3)
key = out[:, 1] & 0xFFFFFFFF
idx = out[:, 0]
assert bool((key[1:] >= key[:-1]).all()), "order"
same = key[1:] == key[:-1]
assert bool((idx[1:][same] > idx[:-1][same]).all()), "stability"
assert torch.equal(torch.sort(idx).values, torch.arange(n, device="cuda")), "permutation"
print(f"4 passes {min(times):.2f} ms (all {[round(t, 2) for t in times]}) VALID", flush=True)
