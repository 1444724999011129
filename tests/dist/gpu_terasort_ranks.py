"""Multi-rank TeraSort through the query API on GPU ranks (run by tests/test_gpu_multirank.py
with DRYAD_DIST_BACKEND=gloo so two ranks can share one GPU): sampling, separators, range_dest,
partition pass, packed all-to-all-v, hybrid local sort with rank hi-bounds, validation."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.models.terasort import TeraSortConfig, TeraSortQueryJob  # noqa: E402
from dryad_amd.parallel.comm import init_world, shutdown  # noqa: E402


def main():
    w = init_world(device="cuda")
    job = TeraSortQueryJob(TeraSortConfig(records_per_rank=int(os.environ.get("TS_RECORDS", "2000000"))), w)
    expect = job.input_checksum()
    for _ in range(2):
        job.step()
        v = job.validate(*expect)
        assert v["ok"], (w.rank, v)
    rep = job.executor_report()
    assert "sort" not in {op for _, op, _ in rep["fallbacks"]}, rep["fallbacks"]
    # a GroupBy with a cross shuffle and a join on device tables across ranks
    import dryad_amd as D
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = w.size
    src = "gen://records64?count=200000&partitions=%d&keys=1000&seed=3" % w.size
    got = sorted(g.FromStore(src).GroupBy(lambda r: r[0], lambda k, gr: (k, gr.Count(), gr.Sum(lambda r: r[1]))))
    l = D.DryadLinqContext(1)
    l.LocalDebug = True
    exp = sorted(l.FromStore(src).GroupBy(lambda r: r[0], lambda k, gr: (k, gr.Count(), gr.Sum(lambda r: r[1]))))
    assert got == exp
    fb = {op for _, op, _ in g._get_executor().last_result["fallbacks"]}
    assert "group_partial" not in fb and "group_final" not in fb, fb
    # OrderBy(k).GroupBy(k) with heavily duplicated keys: GroupBy elides its shuffle, so the fused
    # distributed OrderBy must keep equal keys on one rank (planner keep_ties)
    ts = "gen://terasort?records=200000&partitions=%d&seed=5" % w.size
    k1 = lambda r: r[0:1]  # noqa: E731
    got = sorted(g.FromStore(ts).OrderBy(k1).GroupBy(k1, lambda k, gr: (k, gr.Count())))
    exp = sorted(l.FromStore(ts).OrderBy(k1).GroupBy(k1, lambda k, gr: (k, gr.Count())))
    assert got == exp, (len(got), len(exp))
    assert len(got) == 256
    # skew: every key equal -> the (key, rank, row) tie-break still balances the ranks
    from dryad_amd.ops import recordsort as RS
    n = 300_000
    bufs = RS.SortBuffers.allocate(n, 16, w.device, slack=0.05)
    bufs.rows_in[:n].fill_(7)
    bufs.rows_in[:n, 8:] = torch.randint(0, 256, (n, 8), dtype=torch.uint8, device=w.device)
    st = RS.SortStats()
    out = RS.distributed_sort_rows(bufs, n, 0, 8, w, stats=st)
    assert abs(st.n_out - n) <= 0.05 * n, (w.rank, st.n_out)
    assert torch.equal(out[:, :8], torch.full_like(out[:, :8], 7))
    # uneven inputs per rank through the pipelined exchange (several key sub-ranges per rank):
    # checksum, record count, in-rank order and cross-rank boundaries
    from dryad_amd.ops import terasort as TS
    from dryad_amd.parallel import shuffle
    for subs in (0, 3):
        RS.PIPE_SUBS = subs
        n = 150_000 if w.rank == 0 else 40_000
        bufs = RS.SortBuffers.allocate(190_000, 100, w.device)
        TS.generate(bufs.rows_in[:n], w.rank * 1_000_000, 99)
        acc_in = TS.check(bufs.rows_in[:n]).clone()
        st = RS.SortStats()
        out = RS.distributed_sort_rows(bufs, n, 0, 10, w, stats=st)
        assert st.rounds == (RS.pipeline_subs(150_000 * 100, w.size) if subs == 0 else subs), st.rounds
        acc_out = TS.check(out)
        tot = torch.stack([acc_in[0], acc_out[0], acc_out[1], torch.tensor(out.shape[0], device=w.device)])
        shuffle.all_reduce_(tot, "sum", w)
        assert int(tot[0]) == int(tot[1]) and int(tot[2]) == 0 and int(tot[3]) == 190_000, tot.tolist()
        ends = torch.zeros((1, 20), dtype=torch.uint8, device=w.device)
        ends[0, :10], ends[0, 10:] = out[0, :10], out[-1, :10]
        allends = shuffle.all_gather_tensor(ends, w).cpu().numpy()
        for r in range(w.size - 1):
            assert bytes(allends[r, 10:]) <= bytes(allends[r + 1, :10]), r
    RS.PIPE_SUBS = 0
    # grace hash join across ranks: rank split + all-to-all-v, bucket stores, fused probe; once in
    # HBM and once with a budget that spills buckets to pinned host memory
    from dryad_amd.models.hashjoin import HashJoinConfig, HashJoinJob
    # (pruned rows are 16 of 64 bytes: the pruned spill case needs the smaller budget)
    for budget, prune in ((None, True), (1 << 24, False), (1 << 21, True)):
        job = HashJoinJob(w, HashJoinConfig(rows_r=200_000, rows_s=300_000, chunk_rows=50_000, hbm_budget=budget,
                                            prune=prune))
        res = job.step()
        assert res == job.expected() and res[0] == 300_000, (w.rank, res)
        assert (job.last["spilled_bytes"] > 0) == (budget is not None), job.last
        job.release()
    # out-of-core sort across ranks: one all-to-all-v per chunk round, buckets spilled to pinned host
    # memory and sorted bucket by bucket; checksum, count, in-rank order and rank boundaries
    import numpy as np
    from dryad_amd.ops import extsort as EX
    m64 = (1 << 64) - 1
    s64 = lambda v: (v & m64) - (1 << 64) if (v & m64) >= (1 << 63) else (v & m64)  # noqa: E731
    n = 300_000 if w.rank == 0 else 200_000
    st = EX.ExtSortStats()
    out = EX.external_sort(EX.GenTeraSortSource(w.rank * 1_000_000, n, 99), 0, 10, w, budget=16 << 20, stats=st)
    assert st.chunks > 1 and st.buckets > 1, st
    h, bad, first, last = EX.check_terasort_host(out, 100_000)
    rows = torch.empty((n, 100), dtype=torch.uint8, device=w.device)
    TS.generate(rows, w.rank * 1_000_000, 99)
    hin = int(TS.check(rows)[0].item())
    del rows
    tot = torch.tensor([s64(hin), s64(h), out.n, bad], dtype=torch.int64, device=w.device)
    shuffle.all_reduce_(tot, "sum", w)
    assert int(tot[0]) == int(tot[1]) and int(tot[2]) == 500_000 and int(tot[3]) == 0, tot.tolist()
    ends = torch.zeros((1, 20), dtype=torch.uint8, device=w.device)
    ends[0, :10] = torch.frombuffer(bytearray(first), dtype=torch.uint8)
    ends[0, 10:] = torch.frombuffer(bytearray(last), dtype=torch.uint8)
    allends = shuffle.all_gather_tensor(ends, w).cpu().numpy()
    for r in range(w.size - 1):
        assert bytes(allends[r, 10:]) <= bytes(allends[r + 1, :10]), r
    # keep_ties: every run of equal keys stays on one rank (a following GroupBy skips its shuffle)
    from dryad_amd.io.hosttable import HostRows
    g = np.random.default_rng(w.rank + 1)
    a = g.integers(0, 256, size=(120_000, 16), dtype=np.uint8)
    a[:, :10] = g.integers(0, 5, size=(120_000, 1), dtype=np.uint8)
    out = EX.external_sort(EX.HostRowsSource(HostRows.from_tensor(torch.from_numpy(a), 0, 10)), 0, 10, w,
                           budget=2 << 20, keep_ties=True)
    mine = sorted({bytes(r) for r in out.rows[:, :10].numpy()})
    got = [None] * w.size
    import torch.distributed as dist
    dist.all_gather_object(got, mine)
    seen = [k for ks in got for k in ks]
    assert len(seen) == len(set(seen)) and len(seen) == 5, got
    cnt = torch.tensor([out.n], dtype=torch.int64, device=w.device)
    shuffle.all_reduce_(cnt, "sum", w)
    assert int(cnt) == 120_000 * w.size
    # a gen://terasort read feeding only a distributed OrderBy is generated lazily (entries only);
    # with a key the fused sort cannot take (not a byte-string slice) the records must be
    # materialised before the ordinary sample / range-partition path reads them
    ts = "gen://terasort?records=60000&partitions=%d&seed=21" % w.size
    kint = lambda r: r[3] * 256 + r[4]  # noqa: E731
    gctx = D.DryadLinqContext(platform="gpu")
    gctx.PartitionCount = w.size
    lctx = D.DryadLinqContext(1)
    lctx.LocalDebug = True
    got = list(gctx.FromStore(ts).OrderBy(kint).Select(lambda r: r[0:10]))
    exp = list(lctx.FromStore(ts).OrderBy(kint).Select(lambda r: r[0:10]))
    assert [kint(bytes(x) + bytes(90)) for x in got] == [kint(bytes(x) + bytes(90)) for x in exp]
    assert sorted(map(bytes, got)) == sorted(map(bytes, exp))
    fb = {op for _, op, _ in gctx._get_executor().last_result["fallbacks"]}
    assert not fb & {"sample", "separators", "range_partition", "sort"}, fb
    w.barrier()
    if w.rank == 0:
        print("MULTIRANK_OK", w.size, flush=True)
    torch.cuda.synchronize()
    shutdown()


if __name__ == "__main__":
    main()
