"""Grace hash join (HBM -> pinned host spill) vs the answer derived from the probe table."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _world():
    from dryad_amd.parallel.comm import World
    return World(0, 1, 0, torch.device("cuda", 0), None)


@pytest.mark.parametrize("budget", [None, 1 << 26, 1 << 20])    # in HBM / hybrid / everything spilled
def test_grace_join_matches_expected(budget):
    from dryad_amd.models.hashjoin import HashJoinConfig, HashJoinJob
    cfg = HashJoinConfig(rows_r=300_000, rows_s=450_000, chunk_rows=100_000, hbm_budget=budget)
    job = HashJoinJob(_world(), cfg)
    res = job.step()
    assert res == job.expected()
    assert res[0] == 450_000
    total = (300_000 + 450_000) * 64
    if budget is None:
        assert job.last["in_hbm"] and job.last["spilled_bytes"] == 0
    elif budget == 1 << 26:
        assert not job.last["in_hbm"] and 0 < job.last["spilled_bytes"] < total and job.last["buckets"] > 1
    else:
        assert job.last["spilled_bytes"] == total
    assert job.step() == res        # buffers re-created / released across steps


def test_sort_merge_join_pairs_many_to_many():
    from dryad_amd.ops import grace as G
    l = torch.zeros((6, 16), dtype=torch.uint8, device="cuda")
    r = torch.zeros((5, 16), dtype=torch.uint8, device="cuda")
    lk = [3, 1, 3, 7, 9, 1]
    rk = [1, 3, 3, 8, 1]
    for i, k in enumerate(lk):
        l[i, 0] = k
    for i, k in enumerate(rk):
        r[i, 0] = k
    oo, ii = G.sort_merge_join_pairs(l, r, 0, 8)
    got = sorted(zip(oo.tolist(), ii.tolist()))
    exp = sorted((a, b) for a in range(6) for b in range(5) if lk[a] == rk[b])
    assert got == exp
