"""TeraSort input rows at a 128-byte pitch (one aligned HBM line per record): generator, compact
sort + fix-up gather from padded rows, the exact full-key LSD chain for duplicated keys, and the
one-rank query path that uses them -- against the back-to-back (100-byte pitch) path and numpy."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _gen(n, seed=7):
    from dryad_amd.ops import terasort as TS
    plain = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    kp = torch.empty(n, dtype=torch.int64, device="cuda")
    TS.generate_with_keys64(plain, 0, seed, kp)
    padded = torch.full((n, 128), 0xAB, dtype=torch.uint8, device="cuda")
    kq = torch.empty(n, dtype=torch.int64, device="cuda")
    TS.generate_with_keys64_pitch128(padded, 0, seed, kq)
    return plain, kp, padded, kq


def test_pitch128_generator_matches_plain_rows_and_keys():
    plain, kp, padded, kq = _gen(100_003)
    assert torch.equal(padded[:, :100], plain)
    assert int(padded[:, 100:].count_nonzero()) == 0
    assert torch.equal(kq, kp)


@pytest.mark.parametrize("n", [2, 5000, 300_001])
def test_pitch128_sort_matches_plain_compact_sort(n):
    from dryad_amd.ops import sort as S
    plain, kp, padded, kq = _gen(n, seed=n)
    out_a = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    ref = S.sort_rows_compact(plain, out_a, kp, torch.empty(n, dtype=torch.int64, device="cuda"), 0, 10,
                              hi_bounds=(0, (1 << 64) - 1), keys_ready=True)
    out_b = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    info = {}
    got = S.sort_rows_pitch128(padded, out_b, kq, 0, 10, stats=info)
    assert "pitch128" in info["path"]
    assert torch.equal(got, ref)


def _reference_order(rows: np.ndarray, key_off: int, key_len: int) -> np.ndarray:
    keys = rows[:, key_off:key_off + key_len]
    return np.lexsort(tuple(keys[:, j] for j in range(key_len - 1, -1, -1)))   # stable


@pytest.mark.parametrize("key_off,key_len", [(0, 10), (3, 6), (0, 16)])
def test_pitch128_full_key_chain_with_duplicated_keys(key_off, key_len):
    """Long runs of equal 32-bit windows (the gather's fix-up overflows) and equal full keys: the
    LSD chain of compact sorts over every window gives the stable memcmp order."""
    from dryad_amd.ops import sort as S
    n = 70_000
    g = np.random.default_rng(key_off * 31 + key_len)
    rows = g.integers(0, 256, size=(n, 100), dtype=np.uint8)
    rows[:, key_off:key_off + 4] = 9                                   # every row ties on the first window
    rows[:, key_off + key_len - 1] = g.integers(0, 3, size=n)          # few distinct keys -> long equal runs
    padded = torch.zeros((n, 128), dtype=torch.uint8, device="cuda")
    padded[:, :100] = torch.from_numpy(rows).cuda()
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    out = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    info = {}
    got = S.sort_rows_pitch128(padded, out, keys, key_off, key_len, keys_ready=False, stats=info)
    assert "LSD chain" in info["path"]
    np.testing.assert_array_equal(got.cpu().numpy(), rows[_reference_order(rows, key_off, key_len)])


def test_pitch128_gather_overflow_falls_back_to_the_chain():
    """Keys from the generator but a fix-up overflow (a run of > 64 equal windows): the chain."""
    from dryad_amd.ops import sort as S
    n = 20_000
    plain, kp, padded, kq = _gen(n, seed=3)
    padded[:, 0:4] = 0x11                                              # all rows share the window
    kq.copy_((torch.full((n,), 0x11111111, dtype=torch.int64, device="cuda") << 32)
             | torch.arange(n, dtype=torch.int64, device="cuda"))
    rows = padded[:, :100].cpu().numpy()
    out = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    info = {}
    got = S.sort_rows_pitch128(padded, out, kq, 0, 10, stats=info)
    assert "LSD chain" in info["path"]
    np.testing.assert_array_equal(got.cpu().numpy(), rows[_reference_order(rows, 0, 10)])


def test_one_rank_terasort_query_uses_the_line_aligned_input():
    import dryad_amd as D
    from dryad_amd.ops import terasort as TS
    from dryad_amd.io.providers import provider_for
    n = 1_000_000                                   # 100 MB: large enough for the pooled sets
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = 1
    src = f"gen://terasort?records={n}&partitions=1&seed=11"
    ctx.FromStore(src).OrderBy(lambda r: r[0:10]).ToStore("hbm://ts_pitch", delete_if_exists=True).SubmitAndWait()
    ex = ctx._get_executor()
    runner_path = getattr(ex, "last_sort_path", None)
    out = provider_for("hbm://ts_pitch").get("hbm://ts_pitch")["local"][0].rows
    inp = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    TS.generate(inp, 0, 11)
    h_in = TS.check(inp)
    h_out = TS.check(out)
    torch.cuda.synchronize()
    assert out.shape == (n, 100)
    assert int(h_out[0]) == int(h_in[0]) and int(h_out[1]) == 0
    assert runner_path is not None and "pitch128" in runner_path
    assert ex.last_result["fallbacks"] == []
    provider_for("hbm://ts_pitch").delete("hbm://ts_pitch")


def test_pitch128_gather_fixup_short_runs():
    """Short runs of equal 32-bit windows (about 4 rows each, resolved by the gather's in-LDS
    fix-up) copied by the 16-byte nontemporal-load gather: numpy order."""
    from dryad_amd.ops import sort as S
    n = 200_003
    g = np.random.default_rng(5)
    rows = g.integers(0, 256, size=(n, 100), dtype=np.uint8)
    win = (g.integers(0, 50_000, size=n, dtype=np.uint64) * 85_899).astype(np.uint32)   # spread: top 24 bits differ
    rows[:, 0:4] = win.astype(">u4").view(np.uint8).reshape(n, 4)
    padded = torch.zeros((n, 128), dtype=torch.uint8, device="cuda")
    padded[:, :100] = torch.from_numpy(rows).cuda()
    keys = ((torch.from_numpy(win.astype(np.int64)) << 32) | torch.arange(n, dtype=torch.int64)).cuda()
    out = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    info = {}
    got = S.sort_rows_pitch128(padded, out, keys, 0, 10, keys_ready=True, stats=info)
    assert "LSD chain" not in info["path"], info
    np.testing.assert_array_equal(got.cpu().numpy(), rows[_reference_order(rows, 0, 10)])


def _bucket_gather(padded, e_sorted, key_off, key_len, win):
    from dryad_amd.ops import _lib
    from dryad_amd.ops._lib import c_u32, c_u64, ptr, stream_of
    n = padded.shape[0]
    out = torch.zeros((n, 100), dtype=torch.uint8, device="cuda")
    flags = torch.zeros(2, dtype=torch.int32, device="cuda")
    _lib.call("dr_gather_bucket_pitch128", ptr(padded), ptr(out), ptr(e_sorted), c_u64(n), c_u32(key_off),
              c_u32(key_len), 64 - win, ptr(flags[:1]), ptr(flags[1:]), stream_of(padded))
    return out, int(flags[0].item())


@pytest.mark.parametrize("case", ["random", "ties", "key_off"])
def test_bucket_gather_orders_each_run_by_the_full_key(case):
    """dr_gather_bucket_pitch128: entries sorted on their top 16 window bits only (runs of ~40
    rows), every run ordered in LDS by the rest of the key, ties by position -- numpy's stable
    lexsort of the key bytes."""
    from dryad_amd.ops import sort as S
    n = 40 << 16
    key_off, key_len = (5, 12) if case == "key_off" else (0, 10)
    g = np.random.default_rng({"random": 1, "ties": 2, "key_off": 3}[case])
    rows = g.integers(0, 256, size=(n, 100), dtype=np.uint8)
    if case == "ties":          # few distinct sub-keys per run: the full-key / position tie path
        rows[:, key_off + 2:key_off + key_len] = g.integers(0, 2, size=(n, 1), dtype=np.uint8)
        rows[:, key_off + key_len - 1] = g.integers(0, 3, size=n)
    padded = torch.zeros((n, 128), dtype=torch.uint8, device="cuda")
    padded[:, :100] = torch.from_numpy(rows).cuda()
    e = S.extract_keys64(padded, key_off, key_len, 0, torch.empty(n, dtype=torch.int64, device="cuda"))
    tmp = torch.empty_like(e)
    srt = S.sort_entries64(e, tmp, 16, lookback=False)
    out, ovf = _bucket_gather(padded, srt, key_off, key_len, 16)
    assert ovf == 0
    np.testing.assert_array_equal(out.cpu().numpy(), rows[_reference_order(rows, key_off, key_len)])


def test_bucket_gather_flags_a_run_past_its_window():
    from dryad_amd.ops import sort as S
    n = 1 << 16
    rows = np.random.default_rng(5).integers(0, 256, size=(n, 100), dtype=np.uint8)
    rows[: n // 2, 0:2] = 7                      # one run of 32768 rows on the top 16 bits
    padded = torch.zeros((n, 128), dtype=torch.uint8, device="cuda")
    padded[:, :100] = torch.from_numpy(rows).cuda()
    e = S.extract_keys64(padded, 0, 10, 0, torch.empty(n, dtype=torch.int64, device="cuda"))
    srt = S.sort_entries64(e, torch.empty_like(e), 16, lookback=False)
    _, ovf = _bucket_gather(padded, srt, 0, 10, 16)
    assert ovf & 1


@pytest.mark.parametrize("fmt", ["e64", "e64@out"])
def test_pitch128_bucket_sort_path_matches_the_compact_sort(fmt, monkeypatch):
    """sort_rows_pitch128's bucket path (three look-back passes on 24 bits + the bucket gather),
    entries from the generator in ent_a or in the output's memory, against the plain compact sort."""
    from dryad_amd.ops import sort as S
    from dryad_amd.ops import terasort as TS
    monkeypatch.setattr(S, "BUCKET_MIN_ROWS", 1)
    n = 3 << 24
    plain, kp, padded, kq = _gen(n, seed=11)
    ref = S.sort_rows_compact(plain, torch.empty((n, 100), dtype=torch.uint8, device="cuda"), kp,
                              torch.empty(n, dtype=torch.int64, device="cuda"), 0, 10,
                              hi_bounds=(0, (1 << 64) - 1), keys_ready=True).clone()
    del plain, kp
    out = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    keys = torch.empty(n, dtype=torch.int64, device="cuda")
    home = keys if fmt == "e64" else out.view(-1)[: n * 8].view(torch.int64)
    TS.generate_with_keys64_pitch128(padded, 0, 11, home, torch.tensor([-1, 0], dtype=torch.int64, device="cuda"),
                                     hist=True)
    info = {}
    got = S.sort_rows_pitch128(padded, out, keys, 0, 10, keys_ready=True, stats=info, keys_fmt=fmt)
    assert "bucket sort" in info["path"] and "chain" not in info["path"], info
    assert "gen-hist" in info["path"], info
    assert torch.equal(got, ref)
