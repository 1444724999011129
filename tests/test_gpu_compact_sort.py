"""Compact row sort (8-byte window entries + run fix-up inside the row gather,
csrc/kernels/sort.hip dr_extract_keys64 / dr_sort_u64 / dr_gather_fixup) against a numpy
stable lexicographic sort of the key bytes."""
import numpy as np
import pytest
import torch

from dryad_amd.ops import recordsort as RS
from dryad_amd.ops import sort as S
from dryad_amd.ops import terasort as TS

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref_order(rows: np.ndarray, off: int, ln: int) -> np.ndarray:
    k = rows[:, off:off + ln]
    return np.lexsort(tuple(k[:, j] for j in reversed(range(ln))))


def _sort(rows_t, off, ln, hi_bounds=None, keys_ready=False, ent=None):
    n, stride = rows_t.shape
    out = torch.empty_like(rows_t)
    ent = ent if ent is not None else torch.empty(n, dtype=torch.int64, device=DEV)
    tmp = torch.empty(n, dtype=torch.int64, device=DEV)
    st = {}
    r = S.sort_rows_compact(rows_t, out, ent, tmp, off, ln, hi_bounds=hi_bounds, keys_ready=keys_ready, stats=st)
    return r, st


@pytest.mark.parametrize("n,stride,off,ln", [(1000, 16, 0, 8), (200_003, 100, 0, 10), (70_000, 32, 4, 12),
                                             (50_000, 20, 2, 3), (100_000, 24, 5, 16), (3, 8, 0, 1)])
def test_random_keys(n, stride, off, ln):
    g = torch.Generator().manual_seed(n)
    rows = torch.randint(0, 256, (n, stride), dtype=torch.uint8, generator=g)
    r, st = _sort(rows.to(DEV), off, ln)
    assert r is not None, st
    ref = rows.numpy()[_ref_order(rows.numpy(), off, ln)]
    assert np.array_equal(r.cpu().numpy(), ref), st


def test_shared_prefix_and_duplicates():
    n = 300_000
    g = torch.Generator().manual_seed(7)
    rows = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
    rows[:, :5] = 0x5A                                  # 40 shared leading key bits
    rows[:, 8] = rows[:, 8] % 4                         # a few duplicates of the whole key
    rows[:, 9:12] = 0
    r, st = _sort(rows.to(DEV), 0, 12)
    assert r is not None, st
    assert "prefix=" in st["path"]
    ref = rows.numpy()[_ref_order(rows.numpy(), 0, 12)]
    assert np.array_equal(r.cpu().numpy(), ref), st


def test_long_runs_overflow_then_full_key_fallback():
    n = 100_000
    rows = torch.zeros((n, 16), dtype=torch.uint8)
    rows[:, 8:] = torch.randint(0, 256, (n, 8), dtype=torch.uint8)     # key 0..7 all equal: one run
    r, st = _sort(rows.to(DEV), 0, 8)
    assert r is None and "overflow" in st["path"]
    # local_sort_rows falls back to the 16-byte hybrid sort and stays stable
    ent_a = torch.empty((n, 2), dtype=torch.int64, device=DEV)
    ent_b = torch.empty_like(ent_a)
    out = torch.empty((n, 16), dtype=torch.uint8, device=DEV)
    got = RS.local_sort_rows(rows.to(DEV), out, ent_a, ent_b, 0, 8)
    assert torch.equal(got.cpu(), rows)


def test_generator_fused_e64_keys():
    n = 1 << 20
    rows = torch.empty((n, 100), dtype=torch.uint8, device=DEV)
    ent = torch.empty(n, dtype=torch.int64, device=DEV)
    rng = torch.tensor([-1, 0], dtype=torch.int64, device=DEV)
    TS.generate_with_keys64(rows, 0, 42, ent, rng)
    ref_e = S.extract_keys64(rows, 0, 10, 0, torch.empty(n, dtype=torch.int64, device=DEV))
    assert torch.equal(ent, ref_e)
    mn, mx = (int(x) & ((1 << 64) - 1) for x in rng.cpu().tolist())
    acc_in = TS.check(rows).clone()
    r, st = _sort(rows, 0, 10, hi_bounds=(mn, mx), keys_ready=True, ent=ent)
    assert r is not None, st
    acc = TS.check(r)
    assert int(acc[1]) == 0 and int(acc[0]) == int(acc_in[0])


@pytest.mark.parametrize("dtype,lo,hi", [(torch.int64, -(1 << 40), -(1 << 40) + (1 << 30)), (torch.int32, -5, 300),
                                         (torch.int64, 7, 8), (torch.int16, -30000, 30000),
                                         (torch.uint8, 0, 256), (torch.int64, 0, 1 << 31)])
def test_int_key_sort_matches_stable_argsort(dtype, lo, hi):
    from dryad_amd.ops import relational as R
    n = 500_000
    col = torch.randint(lo, hi, (n,), dtype=torch.int64).to(dtype).to(DEV)
    srt = R.int_key_sort(col)
    assert srt is not None
    perm = (srt[:, 0] & 0xFFFFFFFF).cpu()
    ref = torch.sort(col.cpu().to(torch.int64), stable=True).indices
    assert torch.equal(perm, ref)
    if dtype == torch.int64:
        assert torch.equal(srt[:, 1].cpu() ^ (-(1 << 63)), col.cpu()[ref])


def test_int_key_sort_declines_wide_spans():
    from dryad_amd.ops import relational as R
    col = torch.tensor([0, 1 << 40, 5], dtype=torch.int64, device=DEV)
    assert R.int_key_sort(col) is None


def _sort64_both(ent: torch.Tensor, win: int):
    """(look-back sort result, per-pass count sort result) of the same E64 entries."""
    n = ent.shape[0]
    a, ta = ent.clone(), torch.empty_like(ent)
    flag = __import__("ctypes").c_int(0)
    ws = S._onesweep_workspace(n, ent.device)
    err = S.lookback_error()
    from dryad_amd.ops import _lib
    _lib.call("dr_sort_u64_onesweep", S.ptr(a), S.ptr(ta), S.c_u64(n), 64 - win, 64, S.ptr(ws), S.c_u64(ws.numel()),
              None, S.c_u32(0), S.ptr(err), S.stream_of(a), __import__("ctypes").byref(flag))
    ra = ta if flag.value else a
    b, tb = ent.clone(), torch.empty_like(ent)
    wsb = S._workspace(n, ent.device)
    _lib.call("dr_sort_u64", S.ptr(b), S.ptr(tb), S.c_u64(n), 64 - win, 64, S.ptr(wsb), S.stream_of(b),
              __import__("ctypes").byref(flag))
    rb = tb if flag.value else b
    assert int(err.item()) == 0, "look-back sort failed"
    return ra, rb


@pytest.mark.parametrize("n,win,kind", [((1 << 20) + 12345, 32, "random"), (3_000_001, 24, "random"),
                                        (2_000_000, 32, "skew"), (5000, 16, "random"), (1 << 22, 32, "one")])
def test_onesweep_sort64_matches_stable_reference(n, win, kind):
    """dr_sort_u64_onesweep (one histogram read + look-back scatter per pass) against a stable
    torch sort of the window bits, and bit-identical to the per-pass count sort."""
    g = torch.Generator().manual_seed(n + win)
    if kind == "random":
        w = torch.randint(0, 1 << 32, (n,), generator=g, dtype=torch.int64)
    elif kind == "skew":             # 90% of the windows share every digit: one bucket per pass takes most
        w = torch.randint(0, 1 << 32, (n,), generator=g, dtype=torch.int64)
        w[torch.rand(n, generator=g) < 0.9] = 0x12345678
    else:                            # every window equal
        w = torch.full((n,), 0xABCDEF01, dtype=torch.int64)
    ent = ((w << 32) | torch.arange(n, dtype=torch.int64)).to(DEV)
    ra, rb = _sort64_both(ent, win)
    key = ((ent >> 32) & 0xFFFFFFFF) >> (32 - win)
    order = torch.sort(key.cpu(), stable=True).indices
    ref = ent.cpu()[order]
    assert torch.equal(ra.cpu(), ref)
    assert torch.equal(rb.cpu(), ref)


def test_pitch128_sort_with_generator_histograms():
    """gen://terasort rows at a 128-byte pitch whose generator also wrote the window histograms:
    the sort uses them (no histogram read) and orders exactly like the plain path."""
    n = (1 << 20) + 4097
    rows = torch.empty((n, 128), dtype=torch.uint8, device=DEV)
    keys = torch.empty(n, dtype=torch.int64, device=DEV)
    out_a = torch.empty((n, 100), dtype=torch.uint8, device=DEV)
    out_b = torch.empty((n, 100), dtype=torch.uint8, device=DEV)
    TS.generate_with_keys64_pitch128(rows, 0, 99, keys, hist=True)
    st = {}
    S.sort_rows_pitch128(rows, out_a, keys, 0, 10, keys_ready=True, stats=st)
    assert "gen-hist" in st["path"], st
    TS.generate_with_keys64_pitch128(rows, 0, 99, keys, hist=False)
    st2 = {}
    S.sort_rows_pitch128(rows, out_b, keys, 0, 10, keys_ready=True, stats=st2)
    assert "gen-hist" not in st2["path"], st2
    assert torch.equal(out_a, out_b)
    chk = TS.check(out_a)
    assert int(chk[1]) == 0



def test_onesweep_refuses_foreign_histograms():
    """Producer histograms that do not count the entries (another producer's) are refused before
    any entry moves: the error flag is set and the caller's fallback sorts correctly."""
    n = (1 << 20) + 999
    g = torch.Generator().manual_seed(11)
    w = torch.randint(0, 1 << 32, (n,), generator=g, dtype=torch.int64)
    ent = ((w << 32) | torch.arange(n, dtype=torch.int64)).to(DEV)
    foreign = torch.zeros(4 * 1024, dtype=torch.int32, device=DEV)    # 4 parts, all-zero counts
    e, tmp = ent.clone(), torch.empty_like(ent)
    err = S.lookback_error()
    S.sort_entries64(e, tmp, 32, gen_hist=foreign, err=err)
    assert int(err.item()) & 2
    assert torch.equal(e, ent)                   # nothing moved
    srt = S.sort_entries64(e, tmp, 32, lookback=False)
    assert torch.equal((srt & 0xFFFFFFFF).cpu(), torch.sort(w, stable=True).indices)


def test_sort_rows_compact_recovers_from_failed_lookback(monkeypatch):
    """A failed look-back sort inside the compact row sort is redone with count + scatter passes."""
    from dryad_amd.ops import terasort as TS
    n = (1 << 20) + 4321
    rows = torch.empty((n, 100), dtype=torch.uint8, device=DEV)
    TS.generate(rows, 0, 3)
    real = S.sort_entries64
    calls = []

    def failing(e, tmp, win, gen_hist=None, err=None, lookback=True):
        calls.append(lookback)
        if lookback and err is not None:
            err.fill_(1)                      # as if a spin had given up (entries scrambled)
            e.copy_(e.flip(0))
            return e
        return real(e, tmp, win, gen_hist, err=err, lookback=lookback)
    monkeypatch.setattr(S, "sort_entries64", failing)
    out = torch.empty_like(rows)
    info = {}
    got = S.sort_rows_compact(rows, out, torch.empty(n, dtype=torch.int64, device=DEV),
                              torch.empty(n, dtype=torch.int64, device=DEV), 0, 10, stats=info)
    assert calls == [True, False] and "look-back failed" in info["path"]
    acc = TS.check(got)
    assert int(acc[1].item()) == 0 and int(acc[0].item()) == int(TS.check(rows)[0].item())


def test_sort_workspace_covers_every_geometry():
    """dr_sort_u128_workspace must hold the count matrix of the finest-grained sort that takes it
    (dr_sort_u64_expand: 4096-entry tiles), not only the E128 passes' 8192-entry geometry."""
    from dryad_amd.ops import _lib
    for n in (1, 5000, 500_000, 3_000_000, 1 << 31):
        g = min((n + 4095) // 4096, 1024)
        assert int(_lib.lib().dr_sort_u128_workspace(n)) >= (256 * g + 1024) * 4, n
