"""Shuffle send-side kernels (csrc/kernels/channel.hip) against plain PyTorch references: the stable
multi-column bucket scatter == a stable argsort by bucket + index_select of every column, and the
string-heap compaction == the concatenation of the selected byte ranges."""
import pytest
import torch

from dryad_amd.ops import channel as CH

pytestmark = pytest.mark.gpu


def _ref_scatter(ent, cols, lut):
    d = ent[:, 1] & 0xFF
    if lut is not None:
        d = lut.to(torch.int64)[d]
    order = torch.sort(d, stable=True).indices
    return [c.index_select(0, order) for c in cols], torch.bincount(d, minlength=256)[:256].cpu()


@pytest.mark.parametrize("n,nb", [(1, 3), (511, 2), (513, 7), (100_000, 8), (2_000_003, 256), (777_777, 37)])
def test_scatter_columns_matches_stable_argsort(n, nb):
    g = torch.Generator(device="cuda").manual_seed(n + nb)
    ent = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    ent[:, 1] = torch.randint(0, nb, (n,), device="cuda", generator=g)
    ent[:, 0] = torch.arange(n, device="cuda")
    cols = [torch.randint(-2**62, 2**62, (n,), device="cuda", generator=g),
            torch.randint(-2**31, 2**31 - 1, (n,), device="cuda", generator=g, dtype=torch.int32),
            torch.randn(n, device="cuda", generator=g, dtype=torch.float64),
            torch.randint(0, 2, (n,), device="cuda", generator=g).bool(),
            torch.randint(-30000, 30000, (n,), device="cuda", generator=g, dtype=torch.int16),
            torch.randn((n, 10), device="cuda", generator=g, dtype=torch.float32),     # 40-byte vectors
            torch.randint(0, 255, (n, 100), device="cuda", generator=g, dtype=torch.uint8)]  # TeraSort rows
    assert CH.kernel_ok(cols)
    lut = None
    if nb <= 16:   # rank-major port order for W = 4: ports p -> (p % 4, p // 4)
        order = sorted(range(256), key=lambda p: (p % 4, p // 4))
        inv = [0] * 256
        for i, p in enumerate(order):
            inv[p] = i
        lut = torch.tensor(inv, dtype=torch.uint8, device="cuda")
    got, cnt = CH.scatter_columns(ent, n, cols, lut)
    exp, ecnt = _ref_scatter(ent, cols, lut)
    assert torch.equal(cnt, ecnt)
    for a, b in zip(got, exp):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n,nb", [(1, 3), (511, 2), (100_000, 8), (2_000_003, 256)])
@pytest.mark.parametrize("kind", ["4xint64", "3xint32", "int64+int32+f32", "8xint32", "int64+int8+3xint64+int16"])
def test_scatter_whole_rows_matches_stable_argsort(n, nb, kind):
    """Dword columns of <= 32 bytes per row in total take pc_scatter_rows_kernel (every dword of a
    tile's rows loaded at once): the same stable order as the per-column kernel."""
    g = torch.Generator(device="cuda").manual_seed(7 * n + nb)
    ent = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    ent[:, 1] = torch.randint(0, nb, (n,), device="cuda", generator=g)
    i64 = lambda: torch.randint(-2**62, 2**62, (n,), device="cuda", generator=g)          # noqa: E731
    i32 = lambda: torch.randint(-2**31, 2**31 - 1, (n,), device="cuda", generator=g, dtype=torch.int32)  # noqa: E731
    cols = {"4xint64": lambda: [i64() for _ in range(4)],
            "3xint32": lambda: [i32() for _ in range(3)],
            "int64+int32+f32": lambda: [i64(), i32(), torch.randn(n, device="cuda", generator=g)],
            "8xint32": lambda: [i32() for _ in range(8)],
            "int64+int8+3xint64+int16": lambda: [
                i64(), torch.randint(-128, 127, (n,), device="cuda", generator=g, dtype=torch.int8), i64(), i64(),
                i64(), torch.randint(-30000, 30000, (n,), device="cuda", generator=g, dtype=torch.int16)]}[kind]()
    got, cnt = CH.scatter_columns(ent, n, cols, None)
    exp, ecnt = _ref_scatter(ent, cols, None)
    assert torch.equal(cnt, ecnt)
    for a, b in zip(got, exp):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n,nb", [(1, 3), (513, 7), (2_000_003, 256), (777_777, 37)])
def test_uint8_ports_match_e128_entries(n, nb):
    """The hash partitioner's compact form (one uint8 port per row) moves every column exactly as
    the 16-byte entries do, with or without a port LUT."""
    g = torch.Generator(device="cuda").manual_seed(7 * n + nb)
    ports = torch.randint(0, nb, (n,), device="cuda", generator=g)
    ent = torch.stack([torch.arange(n, device="cuda"), ports], 1)
    cols = [torch.randint(-2**62, 2**62, (n,), device="cuda", generator=g),
            torch.randint(0, 255, (n, 100), device="cuda", generator=g, dtype=torch.uint8)]
    for lut in (None, torch.randperm(256, device="cuda", generator=g).to(torch.uint8)):
        a, ca = CH.scatter_columns(ent, n, cols, lut)
        b, cb = CH.scatter_columns(ports.to(torch.uint8), n, cols, lut)
        assert torch.equal(ca, cb)
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def test_stable_hash_ports_match_entries():
    from dryad_amd.ops import relational as R
    n = 300_001
    k = torch.randint(-2**40, 2**40, (n,), device="cuda")
    keys = [R.HashKey.column(k)]
    e, _ = R.stable_hash_dest(keys, n, 37, False, k.device)
    p, _ = R.stable_hash_dest(keys, n, 37, False, k.device, ports=True)
    assert p.dtype == torch.uint8 and torch.equal(p.to(torch.int64), e[:, 1])


def test_scatter_columns_cpu_path_matches_gpu():
    n = 50_000
    ent = torch.zeros((n, 2), dtype=torch.int64)
    ent[:, 1] = torch.randint(0, 9, (n,))
    cols = [torch.randint(0, 1 << 40, (n,)), torch.randn(n)]
    a, ca = CH.scatter_columns(ent, n, cols)
    b, cb = CH.scatter_columns(ent.cuda(), n, [c.cuda() for c in cols])
    assert torch.equal(ca, cb)
    for x, y in zip(a, b):
        assert torch.equal(x, y.cpu())


@pytest.mark.parametrize("n", [1, 63, 64, 65, 10_000, 1_000_003])
def test_compact_heap_matches_python(n):
    g = torch.Generator(device="cuda").manual_seed(n)
    ln = torch.randint(0, 40, (n,), device="cuda", generator=g)
    ln[::17] = 0
    heap = torch.randint(0, 255, (int(ln.sum()) * 2 + 100,), device="cuda", generator=g, dtype=torch.uint8)
    off = torch.randint(0, heap.numel() - 40, (n,), device="cuda", generator=g)
    out, doff = CH.compact_heap(heap, off, ln)
    h, o, l_ = heap.cpu(), off.cpu().tolist(), ln.cpu().tolist()
    exp = torch.cat([h[a:a + b] for a, b in zip(o, l_)]) if n else torch.zeros(0, dtype=torch.uint8)
    assert torch.equal(out.cpu(), exp)
    cpu_out, cpu_doff = CH.compact_heap(h, off.cpu(), ln.cpu())
    assert torch.equal(cpu_out, exp) and torch.equal(cpu_doff, doff.cpu())


@pytest.mark.parametrize("nbytes", [1, 15, 16, 4097, (3 << 20) + 5])
def test_copy_wide_between_hbm_and_pinned_host(nbytes):
    """CU copy kernel: HBM -> HBM, page-locked host -> HBM and HBM -> page-locked host (through
    the host buffer's device mapping), tails that are not a multiple of 16 bytes included."""
    from dryad_amd.ops import _lib
    g = torch.Generator().manual_seed(nbytes)
    src_h = _lib.PinnedHostBuffer((nbytes,))
    src_h.tensor.copy_(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g))
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    CH.copy_wide(d, src_h.tensor)
    d2 = torch.empty_like(d)
    CH.copy_wide(d2, d, grid=7)
    back = _lib.PinnedHostBuffer((nbytes,))
    CH.copy_wide(back.tensor, d2)
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), src_h.tensor)
    assert torch.equal(back.tensor, src_h.tensor)
    with pytest.raises(ValueError):
        CH.copy_wide(d[:nbytes - 1] if nbytes > 1 else d[:0], src_h.tensor)
