"""hipGraph replay of launch-bound loops (dryad_amd/runtime/hipgraph.py) against eager runs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _points(n, k, seed=3):
    from dryad_amd.ops import kmeans as KM
    x = KM.generate(torch.empty((n, KM.DIM), dtype=torch.float32, device="cuda"), seed=seed)
    c = x[torch.randperm(n, device="cuda", generator=torch.Generator("cuda").manual_seed(seed))[:k]].clone()
    return x, c


@pytest.mark.parametrize("k", [16, 64])
def test_kmeans_graph_matches_eager(k):
    from dryad_amd.ops import kmeans as KM
    from dryad_amd.runtime.hipgraph import KMeansGraph
    x, c0 = _points(200_003, k)
    c = c0.clone()
    ws = KM.KMeansWorkspace(x.shape[0], k, x.device)
    for _ in range(8):
        s, n, _ = KM.step(x, c, ws)
        c = KM.update(c, s, n)
    g = KMeansGraph(x, c0, unroll=4)
    got = g.run(8)
    torch.cuda.synchronize()
    assert torch.allclose(got, c, rtol=1e-5, atol=1e-5), (got - c).abs().max().item()
    # a replay after restart repeats the trajectory
    g.restart()
    again = g.run(8).clone()
    assert torch.allclose(again, c, rtol=1e-5, atol=1e-5)


def test_graphed_loop_counts_replays():
    from dryad_amd.runtime.hipgraph import GraphedLoop
    acc = torch.zeros(1, dtype=torch.int64, device="cuda")
    loop = GraphedLoop(lambda: acc.add_(1), unroll=5, warmup=2)
    assert int(acc.item()) == 2 + 0          # warmup ran eagerly; capture does not execute
    loop.replay(3)
    assert int(acc.item()) == 2 + 15
