"""W ranks sharing one GPU over gloo (tests/test_gpu_stream_shuffle.py): a GroupBy and a Distinct
over W partitions whose received partials exceed each rank's HBM budget run as the streamed
shuffle (rounds of partial -> hash partition -> exchange -> fold), checked against the LocalDebug
oracle on every rank."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import dryad_amd as D  # noqa: E402
from dryad_amd.parallel.comm import init_world, shutdown  # noqa: E402


def main():
    w = init_world(device="cuda")
    W = w.size
    src = f"gen://records64?count={300_000 * W}&partitions={W}&keys={150_000 * W}&seed=5"
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = W
    g.HbmBudgetBytes = 4 << 20          # the received partials (~4.8 MB per rank) exceed it
    g.StreamChunkBytes = 1 << 20
    g.StreamShuffle = True
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    q = lambda c: c.FromStore(src).Where(lambda r: r[2] % 7 != 1).GroupBy(  # noqa: E731
        lambda r: r[0], lambda k, grp: (k, grp.Count(), grp.Sum(lambda r: r[1]), grp.Max(lambda r: r[3])))
    got = sorted(q(g))
    res = g._get_executor().last_result
    st = [v for v in (res.get("streamed") or {}).values() if v.get("kind") == "streamed shuffle"]
    assert st and st[0]["rounds"] > 2, res.get("streamed")
    assert res["fallbacks"] == [], res["fallbacks"]
    assert got == sorted(q(loc)), "GroupBy differs from the oracle"
    q2 = lambda c: c.FromStore(src).Select(lambda r: r[0] % 90_001).Distinct()  # noqa: E731
    got2 = sorted(q2(g))
    assert got2 == sorted(q2(loc)), "Distinct differs from the oracle"
    # a repartition written to a partfile table as rounds (one part writer per rank)
    out = os.environ.get("SS_TMP", "/tmp") + f"/ss_rep_{W}.pt"
    q3 = lambda c: c.FromStore(src).HashPartition(lambda r: r[1], W).Select(lambda r: (r[1], r[0] * 3))  # noqa: E731
    q3(g).ToStore("partfile://" + out, delete_if_exists=True).SubmitAndWait()
    res3 = g._get_executor().last_result
    st3 = [v for v in (res3.get("streamed") or {}).values() if v.get("kind") == "streamed shuffle"]
    assert st3 and st3[0]["mode"] == "repartition" and st3[0]["result_bytes"] > 0, res3.get("streamed")
    assert res3["fallbacks"] == [], res3["fallbacks"]
    if w.rank == 0:
        assert sorted(loc.FromStore("partfile://" + out)) == sorted(q3(loc)), "repartition differs from the oracle"
    w.barrier()
    print(f"STREAM_SHUFFLE_OK {W} rounds={st[0]['rounds']} exchanged_GB={st[0]['exchanged_GB']}", flush=True)
    shutdown()


if __name__ == "__main__":
    main()
