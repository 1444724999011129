"""k-means MFMA kernel vs plain PyTorch fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,k", [(1, 1), (1000, 7), (50_000, 32), (100_003, 100), (40_000, 200), (20_000, 300), (30_000, 1000), (5_000, 4096)])
def test_kmeans_step_matches_reference(n, k):
    from dryad_amd.ops import kmeans as KM
    x = torch.empty((n, KM.DIM), dtype=torch.float32, device="cuda")
    KM.generate(x, 0, blobs=max(1, k // 2), seed=n)
    c = x[torch.randperm(n, device="cuda")[: min(n, k)]].clone()
    if c.shape[0] < k:
        c = torch.cat([c, torch.randn((k - c.shape[0], KM.DIM), device="cuda")])
    sums, counts, assign = KM.step(x, c)
    rs, rc, ra, d = KM.step_reference(x, c)
    # points whose best and second-best distances are (numerically) tied may legitimately differ
    top2 = torch.topk(d, min(2, k), dim=1, largest=False).values
    gap = (top2[:, 1] - top2[:, 0]) if k > 1 else torch.full((n,), 1e9, device="cuda")
    tied = gap <= 1e-3 * top2[:, 0].abs().clamp_min(1.0)
    mism = (assign.long() != ra.long()) & ~tied
    assert int(mism.sum()) == 0
    if int(tied.sum()) == 0:
        assert torch.equal(counts, rc)
        torch.testing.assert_close(sums, rs, rtol=1e-4, atol=1e-2)
    assert int(counts.sum()) == n


@pytest.mark.parametrize("planes", [True, False])
@pytest.mark.parametrize("n,k", [(1, 1), (1000, 7), (50_003, 64)])
def test_kmeans_step_both_paths_match_reference(n, k, planes):
    """K <= 64: the split-plane kernel (default) and the f32-input kernel agree with the f64 oracle."""
    from dryad_amd.ops import kmeans as KM
    x = torch.empty((n, KM.DIM), dtype=torch.float32, device="cuda")
    KM.generate(x, 0, blobs=max(1, k // 2), seed=n + 7)
    c = x[torch.randperm(n, device="cuda")[:k]].clone()
    if c.shape[0] < k:
        c = torch.cat([c, torch.randn((k - c.shape[0], KM.DIM), device="cuda")])
    sums, counts, assign = KM.step(x, c, planes=planes)
    rs, rc, ra, d = KM.step_reference(x, c)
    top2 = torch.topk(d, min(2, k), dim=1, largest=False).values
    tied = (top2[:, 1] - top2[:, 0] <= 1e-3 * top2[:, 0].abs().clamp_min(1.0)) if k > 1 else torch.zeros(n, dtype=torch.bool, device="cuda")
    assert int(((assign.long() != ra.long()) & ~tied).sum()) == 0
    if int(tied.sum()) == 0:
        assert torch.equal(counts, rc)
        torch.testing.assert_close(sums, rs, rtol=2e-5, atol=1e-3)


def test_kmeans_plane_written_once():
    """The once-per-table state: xh = round-to-nearest bf16 of x, |x| per point, cached across
    steps and rebuilt after an in-place change of the points."""
    from dryad_amd.ops import kmeans as KM
    g = torch.Generator().manual_seed(3)
    x = (torch.randn((4099, KM.DIM), generator=g) * torch.logspace(-20, 20, 4099)[:, None]).cuda()
    sp = KM.split_points(x)
    assert torch.equal(sp.xh, x.bfloat16())
    ok = x.abs().amax(1) < 1e17          # |x|^2 of larger rows overflows f32 (the near-tie bound
    torch.testing.assert_close(sp.xnorm[ok], x[ok].double().norm(dim=1).float(), rtol=1e-5, atol=0)
    big = x.abs().amax(1) > 1e20
    assert bool(torch.isinf(sp.xnorm[big]).all())   # becomes inf: such points are always re-ranked)
    assert KM.split_points(x) is sp                     # cached across steps
    x.mul_(2)
    assert KM.split_points(x) is not sp                 # an in-place change rebuilds it


@pytest.mark.parametrize("planes", [True, False])
def test_kmeans_sums_exact_on_24bit_points(planes):
    """Coordinates using all 24 significand bits (a two-part bf16 split drops their low bits):
    one point per cluster, so the sums must equal the points bit for bit, also after every point
    changes cluster (the kept sums move the exact rows)."""
    from dryad_amd.ops import kmeans as KM
    g = torch.Generator().manual_seed(5)
    k = 64
    x = torch.randint(1 << 23, 1 << 24, (k, KM.DIM), generator=g).float().cuda() * 2.0 ** -20
    h, m, _ = KM.split_reference(x)
    assert not torch.equal(h.float() + m.float(), x)     # the data really needs the third part
    ws = KM.KMeansWorkspace(k, k, x.device)
    sums, counts, assign = KM.step(x, x.clone(), ws, planes=planes)
    assert torch.equal(assign.long().cpu(), torch.arange(k))
    assert torch.equal(counts, torch.ones(k, dtype=torch.int64, device="cuda"))
    assert torch.equal(sums, x.double())
    perm = torch.randperm(k, generator=g)
    sums, counts, assign = KM.step(x, x[perm.cuda()].clone(), ws, planes=planes)
    inv = torch.argsort(perm)
    assert torch.equal(assign.long().cpu(), inv)
    assert torch.equal(sums, x[perm.cuda()].double())


def test_kmeans_planes_iterations_track_f64_sums():
    """Ten iterations on the plane path (assignments change, so rows move between the kept sums):
    every step's sums equal the f64 oracle's up to f64 summation order."""
    from dryad_amd.ops import kmeans as KM
    n, k = 300_000, 48
    x = torch.empty((n, KM.DIM), dtype=torch.float32, device="cuda")
    KM.generate(x, 0, blobs=32, seed=11)
    x.add_(1000.0)                                      # constant offset: xl is far from zero-mean
    c = x[:k].clone()
    ws = KM.KMeansWorkspace(n, k, x.device)
    for _ in range(10):
        s, cnt, a = KM.step(x, c, ws)
        rs, rc, ra, _d = KM.step_reference(x, c)
        if torch.equal(a.long(), ra.long()):
            assert torch.equal(cnt, rc)
            torch.testing.assert_close(s, rs, rtol=1e-12, atol=1e-6)
        c = KM.update(c, s, cnt)


def test_kmeans_generate_counter_based():
    from dryad_amd.ops import kmeans as KM
    a = torch.empty((1000, KM.DIM), dtype=torch.float32, device="cuda")
    b = torch.empty((3000, KM.DIM), dtype=torch.float32, device="cuda")
    KM.generate(a, 2000, 16, 5)
    KM.generate(b, 0, 16, 5)
    assert torch.equal(a, b[2000:])


def test_kmeans_converges_on_blobs():
    from dryad_amd.ops import kmeans as KM
    n, k = 200_000, 16
    x = torch.empty((n, KM.DIM), dtype=torch.float32, device="cuda")
    KM.generate(x, 0, blobs=k, seed=3)
    c = x[:k].clone()
    ws = KM.KMeansWorkspace(n, k, x.device)
    for _ in range(10):
        s, cnt, _a = KM.step(x, c, ws)
        c = KM.update(c, s, cnt)
    _, _, a, d = KM.step_reference(x, c)
    inertia = d.min(1).values + (x * x).sum(1)
    assert float(inertia.mean()) < 1.0   # blobs have per-dim noise 0.2*U(-.5,.5): within-blob MSE ~0.43


@pytest.mark.parametrize("k", [2, 40])
def test_kmeans_mfma_near_ties_rerank_exactly(k):
    """Points just off the bisector of two close centroids: the split-bf16 distance estimate
    cannot order them (its error bound is ~100x the margin), the exact f32 re-rank must."""
    from dryad_amd.ops import kmeans as KM
    g = torch.Generator().manual_seed(1)
    c = (torch.rand((k, KM.DIM), generator=g, dtype=torch.float64) * 10 - 5)
    u = torch.randn(KM.DIM, generator=g, dtype=torch.float64)
    u /= u.norm()
    c[1] = c[0] + u
    n = 4096
    eps = (torch.rand(n, generator=g, dtype=torch.float64) - 0.5) * 0.04
    eps[eps.abs() < 0.004] = 0.004
    x = (c[0] + c[1]) / 2 + eps[:, None] * u[None, :]
    xf, cf = x.float().cuda(), c.float().cuda()
    assert KM.mode(k) == 3
    sums, counts, assign = KM.step(xf, cf)
    d = ((xf.double()[:, None, :] - cf.double()[None, :, :]) ** 2).sum(-1)
    exp = torch.argmin(d, 1)
    assert torch.equal(assign.long().cpu(), exp.cpu())
    assert int(counts.sum()) == n
    ref = torch.zeros((k, KM.DIM), dtype=torch.float64, device="cuda").index_add_(0, exp, xf.double())
    torch.testing.assert_close(sums, ref, rtol=1e-5, atol=1e-3)
