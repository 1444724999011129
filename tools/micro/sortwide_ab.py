"""A/B of the wide-entry sort passes (csrc/kernels/sort.hip dr_sort_wide: rs_scatter_v2 at 256 threads
vs rs_scatter_w, -DDR_SORTW_* variant libraries via DRYAD_KERNEL_LIB) through relational.payload_groups:
n rows, an int64 key uniform over 2^24 values (3 passes of 32-byte E256 entries), Count / Sum / Min /
Max of three int64 columns; checked against torch bincount / index_add / scatter_reduce."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from dryad_amd.ops import relational as R  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
K = 1 << 24
g = torch.Generator(device="cuda").manual_seed(5)
key = torch.randint(0, K, (n,), device="cuda", generator=g, dtype=torch.int64)
v1, v2, v3 = (torch.randint(-1000, 1000, (n,), device="cuda", generator=g, dtype=torch.int64) for _ in range(3))
specs = [("count", None, torch.int64), ("sum", v1, torch.int64), ("min", v2, torch.int64), ("max", v3, torch.int64)]
times = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = R.payload_groups(key, specs)
    torch.cuda.synchronize()
    times.append((time.perf_counter() - t0) * 1e3)
assert got is not None
keys, outs = got
cnt = torch.bincount(key, minlength=K)
present = torch.nonzero(cnt).squeeze(1)
assert torch.equal(keys.to(torch.int64), present), "keys"
assert torch.equal(outs[0].to(torch.int64), cnt[present]), "count"
s = torch.zeros(K, dtype=torch.int64, device="cuda").index_add_(0, key, v1)
assert torch.equal(outs[1].to(torch.int64), s[present]), "sum"
mn = torch.full((K,), 1 << 40, dtype=torch.int64, device="cuda").scatter_reduce_(0, key, v2, "amin")
mx = torch.full((K,), -(1 << 40), dtype=torch.int64, device="cuda").scatter_reduce_(0, key, v3, "amax")
assert torch.equal(outs[2].to(torch.int64), mn[present]) and torch.equal(outs[3].to(torch.int64), mx[present]), "min/max"
print(f"payload_groups {min(times):.2f} ms (all {[round(t, 2) for t in times]}) VALID", flush=True)
