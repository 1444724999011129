"""Streamed shuffle (runtime/stream_shuffle.py): a multi-partition GroupBy / Distinct run as
pipelined rounds (chunk -> partial -> hash partition -> asynchronous exchange -> fold into each
final partition's running state), with received partials far past the HBM budget; and streamed
results written to their store bucket by bucket (runtime/sinks.py).  Against the LocalDebug oracle,
no host fallbacks."""
import os
import subprocess
import sys

import pytest

import dryad_amd as D

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "gen://records64?count={n}&partitions={P}&keys={k}&seed=21"


def _loc():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def _ctx(P, budget=8 << 20, chunk=1 << 20, force=True):
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = P
    c.HbmBudgetBytes = budget
    c.StreamChunkBytes = chunk
    if force is not None:
        c.StreamShuffle = force
    return c


def _shuffle_stats(c):
    r = c._get_executor().last_result
    st = [v for v in (r.get("streamed") or {}).values() if v.get("kind") == "streamed shuffle"]
    return r, st


def _close(got, exp):
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        assert a[:-1] == b[:-1] and abs(a[-1] - b[-1]) <= 1e-9 * max(1.0, abs(b[-1])), (a, b)


@pytest.mark.parametrize("keys,dense", [(5_000, True), (300_000, True), (300_000, False)])
def test_streamed_shuffle_groupby_matches_oracle(keys, dense):
    """Two partitions on one rank: every round's partials exchanged (to itself) and folded into the
    final partitions' running states (dense by key, or hash buckets spilled past the 8 MB budget)."""
    src = SRC.format(n=800_000, P=2, k=keys)
    q = lambda c: c.FromStore(src).Where(lambda r: r[3] % 5 != 0).GroupBy(  # noqa: E731
        lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Min(lambda r: r[2]),
                                      g.Max(lambda r: r[4]), g.Average(lambda r: r[5])))
    g = _ctx(2)
    g.StreamDenseState = dense
    got = sorted(q(g))
    res, st = _shuffle_stats(g)
    assert st and st[0]["rounds"] > 4 and st[0]["received_rows"] > 0, st
    assert res["fallbacks"] == [], res["fallbacks"]
    if not dense and keys > 100_000:
        assert st[0]["spilled_bytes"] > 0, st
    _close(got, sorted(q(_loc())))


def test_streamed_shuffle_holds_received_partials_and_reduces_once():
    """A budget the received partials fit: every round is held in HBM and each final partition
    reduces them ONCE after the last round (the bulk stage's kernels), no per-round folds."""
    src = SRC.format(n=600_000, P=2, k=40_000)
    q = lambda c: c.FromStore(src).GroupBy(lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]),  # noqa: E731
                                                                          g.Max(lambda r: r[4])))
    g = _ctx(2, budget=1 << 30)
    got = sorted(q(g))
    res, st = _shuffle_stats(g)
    assert st and st[0]["rounds"] > 2 and st[0]["held_batches"] == 2 and st[0]["spilled_bytes"] == 0, st
    assert res["fallbacks"] == [], res["fallbacks"]
    assert got == sorted(q(_loc()))


def test_streamed_shuffle_distinct_to_host_table():
    """Distinct over two partitions, the result streamed bucket by bucket into pinned host columns
    (host://), read back oracle-equal."""
    src = SRC.format(n=600_000, P=2, k=1 << 22)
    q = lambda c: c.FromStore(src).Select(lambda r: r[0] % 400_003).Distinct()  # noqa: E731
    g = _ctx(2)
    q(g).ToStore("host://ss_distinct", delete_if_exists=True).SubmitAndWait()
    res, st = _shuffle_stats(g)
    assert st and st[0]["result"] == "streamed to the output store", st
    assert res["fallbacks"] == [], res["fallbacks"]
    got = sorted(g.FromStore("host://ss_distinct"))
    assert got == sorted(q(_loc()))


@pytest.mark.parametrize("P,store", [(2, "host"), (1, "partfile")])
def test_streamed_repartition_to_store(P, store, tmp_path):
    """HashPartition -> Select -> ToStore as rounds: each received round through B's Select and
    straight into the output sink, never a whole partition in HBM; oracle-equal."""
    src = SRC.format(n=500_000, P=P, k=1 << 20)
    uri = "host://ss_rep" if store == "host" else "partfile://" + str(tmp_path / "rep.pt")
    q = lambda c: c.FromStore(src).Where(lambda r: r[2] % 3 != 0).HashPartition(lambda r: r[0], P).Select(  # noqa: E731
        lambda r: (r[0], r[1] + r[3]))
    g = _ctx(P)
    q(g).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    res, st = _shuffle_stats(g)
    assert st and st[0]["mode"] == "repartition" and st[0]["rounds"] > 4, st
    assert st[0]["result"] == "streamed to the output store" and st[0]["result_bytes"] > 0, st
    assert res["fallbacks"] == [], res["fallbacks"]
    assert sorted(g.FromStore(uri)) == sorted(q(_loc()))


def test_streamed_groupby_result_to_partfile(tmp_path):
    """A leaf streamed GroupBy (one partition past the budget) writes its buckets' results straight
    into the output part files (PartFileSplitBytes: several at once) instead of concatenating them."""
    src = SRC.format(n=500_000, P=1, k=200_000)
    uri = "partfile://" + str(tmp_path / "g.pt")
    q = lambda c: c.FromStore(src).GroupBy(lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1])))  # noqa
    g = _ctx(1, budget=16 << 20, force=None)
    g.StreamDenseState = False
    g.PartFileSplitBytes = 1
    q(g).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    r = g._get_executor().last_result
    st = [v for v in (r.get("streamed") or {}).values() if v.get("kind") == "streamed aggregation"]
    assert st and st[0]["result"] == "streamed to the output store" and st[0]["result_bytes"] > 0, st
    assert r["fallbacks"] == [], r["fallbacks"]
    assert sorted(g.FromStore(uri)) == sorted(q(_loc()))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("ranks", [2, 8])
def test_streamed_shuffle_ranks_share_one_gpu(ranks, tmp_path):
    """W gloo ranks on one GPU: a GroupBy and a Distinct whose received partials exceed every
    rank's HBM budget run as the streamed shuffle, oracle-equal (tests/dist/gpu_stream_shuffle_ranks.py)."""
    env = dict(os.environ, DRYAD_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                          "--master-addr", "127.0.0.1", "--master-port", str(29740 + ranks),
                          os.path.join(ROOT, "tests", "dist", "gpu_stream_shuffle_ranks.py")],
                         capture_output=True, text=True, timeout=860, env=env, cwd=ROOT)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert f"STREAM_SHUFFLE_OK {ranks}" in out.stdout
