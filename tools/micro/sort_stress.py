"""Exactness stress of the count-matrix radix sorts over many sizes (partial tiles, few workgroups,
the 1024-workgroup cap): dr_sort_u128 (sort_entries), dr_sort_u64 (sort_entries64 without the
look-back), dr_sort_u64_expand (int_key_sort) and dr_sort_wide (payload_groups) against torch
stable sorts.  Run with DRYAD_KERNEL_LIB pointing at a variant library to check its kernels."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from dryad_amd.ops import relational as R  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402

SIZES = [2, 63, 64, 65, 1000, 2047, 2048, 2049, 8191, 8192, 8193, 20000, 123457, 1 << 20, 3_000_001, 9_000_011,
         40_000_003]
g = torch.Generator(device="cuda").manual_seed(11)
bad = []
for n in SIZES:
    # E128: lo = index, hi = random 40-bit; sort on hi bits [64, 104)
    e = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    e[:, 0] = torch.arange(n, device="cuda")
    e[:, 1] = torch.randint(0, 1 << 40, (n,), device="cuda", generator=g)
    ref = torch.sort(e[:, 1], stable=True).indices
    out = S.sort_entries(e.clone(), 64, 104)
    if not torch.equal(out[:, 0], ref):
        bad.append(("u128", n))
    # E64 count-matrix sort of the top 24 bits
    v = (torch.randint(0, 1 << 31, (n,), device="cuda", generator=g) << 33) | torch.arange(n, device="cuda")
    o64 = S.sort_entries64(v.clone(), torch.empty_like(v), 24, lookback=False)
    ref64 = torch.sort((v >> 40) & 0xFFFFFF, stable=True).indices
    if not torch.equal(o64 & ((1 << 33) - 1), ref64):
        bad.append(("u64", n))
    # expand sort of an int key of span 2^20
    k = torch.randint(-(1 << 19), 1 << 19, (n,), device="cuda", generator=g)
    srt = R.int_key_sort(k)
    if srt is None or not torch.equal(srt[:, 0] & 0xFFFFFFFF, torch.sort(k, stable=True).indices):
        bad.append(("expand", n))
    # wide-entry sort through payload_groups (key span 2^18, 3 passes)
    kk = torch.randint(0, 1 << 18, (n,), device="cuda", generator=g)
    vv = torch.randint(-50, 50, (n,), device="cuda", generator=g)
    got = R.payload_groups(kk, [("count", None, torch.int64), ("sum", vv, torch.int64)])
    if got is not None:
        cnt = torch.bincount(kk, minlength=1 << 18)
        pres = torch.nonzero(cnt).squeeze(1)
        sm = torch.zeros(1 << 18, dtype=torch.int64, device="cuda").index_add_(0, kk, vv)
        if not (torch.equal(got[0].to(torch.int64), pres) and torch.equal(got[1][0].to(torch.int64), cnt[pres])
                and torch.equal(got[1][1].to(torch.int64), sm[pres])):
            bad.append(("wide", n))
    torch.cuda.synchronize()
    print(f"n={n} done, failures so far {bad}", flush=True)
print("STRESS", "OK" if not bad else f"FAIL {bad}", flush=True)
