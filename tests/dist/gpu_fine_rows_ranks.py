"""Multi-rank OrderBy over MATERIALISED tables through the fine-bucket exchange, on GPU ranks that
share one GPU (gloo transport; run by tests/test_gpu_multirank.py):

  * gen://terasort read into a 128-byte-pitch table (the bench default) and the GenFusedShuffle
    variant, through the query API, validated valsort-style;
  * an hbm:// input table (read in place, sorted into a buffer set of its own) and a partfile://
    table of raw rows, both validated;
  * skew: all keys equal with the ties kept (OrderBy(k).GroupBy(k)), so one rank's key range
    overflows its buffer: it receives into larger buffers of its own, and without HBM for them
    every rank stops at the voted capacity check within seconds, instead of blocking in the
    exchange until the collective timeout;
  * heavy duplication with ties split: the fine cut would overflow, the E128 path splits the run.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import dryad_amd as D  # noqa: E402
from dryad_amd.models.terasort import TeraSortConfig, TeraSortQueryJob, TeraSortStoredJob  # noqa: E402
from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402
from dryad_amd.parallel import shuffle  # noqa: E402
from dryad_amd.parallel.comm import init_world, shutdown  # noqa: E402


def _valsort(rows, w, expect_hash, expect_n):
    acc = TS.check(rows)
    cnt = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    shuffle.all_reduce_(acc, "sum", w)
    shuffle.all_reduce_(cnt, "sum", w)
    ends = torch.zeros((1, 21), dtype=torch.uint8, device=rows.device)
    if rows.shape[0]:
        ends[0, 0] = 1
        ends[0, 1:11], ends[0, 11:] = rows[0, :10], rows[-1, :10]
    prev = None
    for r in shuffle.all_gather_tensor(ends, w).cpu().numpy():
        if r[0]:
            assert prev is None or prev <= bytes(r[1:11]), "rank boundary out of order"
            prev = bytes(r[11:])
    assert int(acc[0]) == expect_hash and int(acc[1]) == 0 and int(cnt) == expect_n, (acc.tolist(), int(cnt))


def _rows64(w, base):
    import numpy as np
    from dryad_amd.io.providers import provider_for
    from dryad_amd.runtime.jobmanager import write_schema
    n, W = 250_000, w.size
    g = np.random.default_rng(64)
    rows = g.integers(0, 256, size=(W * n, 64), dtype=np.uint8)
    key = g.integers(0, 1 << 63, size=W * n, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    key[::50] = key[7]                                      # runs of equal keys
    idx = np.arange(W * n, dtype=np.uint64)
    rows[:, 8:16] = key.astype(">u8").view(np.uint8).reshape(-1, 8)
    rows[:, 16:24] = idx.astype(">u8").view(np.uint8).reshape(-1, 8)
    uri = f"partfile://{base}/rows64"
    if w.rank == 0:
        prov = provider_for(uri)
        prov.write_table(uri, [rows[p * n: (p + 1) * n].tobytes() for p in range(W)], None)
        write_schema(prov._path(uri), None, "rows", stride=64, key_off=8, key_len=8)
    w.barrier()
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = W
    for desc in (False, True):
        q = ctx.FromStore(uri)
        q = q.OrderByDescending(lambda r: r[8:16]) if desc else q.OrderBy(lambda r: r[8:16])
        q.ToStore("hbm://rows64_out", delete_if_exists=True).SubmitAndWait()
        res = ctx._get_executor().last_result
        ex = res["exchange"]
        assert ex is not None and "fine-bucket exchange over the table (pitch 64)" in ex["path"], (desc, ex)
        got = provider_for("hbm://rows64_out").get("hbm://rows64_out")["local"][w.rank].rows.cpu().numpy()
        counts = shuffle.all_gather_tensor(torch.tensor([got.shape[0]], dtype=torch.int64, device=w.device), w)
        counts = counts.view(-1).tolist()
        assert sum(counts) == W * n, counts
        order = np.lexsort((idx, ~key if desc else key))
        a = sum(counts[: w.rank])
        assert np.array_equal(got, rows[order[a: a + got.shape[0]]]), (w.rank, desc)


def _records64(w):
    from dryad_amd.io.providers import provider_for
    W, n = w.size, 200_000
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = W
    ctx.FromStore(f"gen://records64?count={W * n}&partitions={W}&keys=5000&seed=9") \
        .ToStore("hbm://r64_in", delete_if_exists=True).SubmitAndWait()
    t = provider_for("hbm://r64_in").get("hbm://r64_in")["local"][w.rank]
    names = list(t.cols)
    mine = torch.stack([t.cols[c][: t.n] for c in names], 1)
    allin = shuffle.all_gather_varlen(mine, w)               # rank order = the ties' order
    for field, desc in (("V1", False), ("Key", True), ("V1", True)):
        q = ctx.FromStore("hbm://r64_in")
        sel = (lambda r: r.V1) if field == "V1" else (lambda r: r.Key)
        q = q.OrderByDescending(sel) if desc else q.OrderBy(sel)
        q.ToStore("hbm://r64_out", delete_if_exists=True).SubmitAndWait()
        ex = ctx._get_executor().last_result["exchange"]
        assert ex is not None and "columns packed into" in ex["path"] and "fine-bucket" in ex["path"], (field, desc, ex)
        o = provider_for("hbm://r64_out").get("hbm://r64_out")["local"][w.rank]
        got = torch.stack([o.cols[c][: o.n] for c in names], 1)
        counts = shuffle.all_gather_tensor(torch.tensor([o.n], dtype=torch.int64, device=w.device), w).tolist()
        assert sum(counts) == W * n, counts
        _, order = torch.sort(allin[:, names.index(field)], descending=desc, stable=True)
        a = sum(counts[: w.rank])
        assert torch.equal(got, allin[order[a: a + o.n]]), (w.rank, field, desc)


def main():
    w = init_world(device="cuda")
    n = int(os.environ.get("TS_RECORDS", "1500000"))
    cfg = TeraSortConfig(records_per_rank=n)
    # 1. the bench's default: the generated table at a 128-byte pitch, fine-bucket exchange over it
    for gen_fused in (False, True):
        job = TeraSortQueryJob(cfg, w, gen_fused=gen_fused)
        expect = job.input_checksum()
        for _ in range(2):
            job.step()
            v = job.validate(*expect)
            assert v["ok"], (w.rank, gen_fused, v)
        ex = job.executor_report()["exchange"]
        want = "records generated into the send rows" if gen_fused else "fine-bucket exchange over the table"
        assert ex is not None and want in ex["path"], ex
        assert ex["rounds"] == len(ex["round_send_MB"]) and ex["send_GB"] > 0, ex
        if not gen_fused:     # the table's send side overlapped with the exchange, round by round
            assert "rounds packed as they go out" in ex["path"] and "first_round_queued_ms" in ex, ex
    # 2. an hbm:// table (a previous job's output) read in place, and a stored partfile of rows
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = w.size
    src = f"gen://terasort?records={n * w.size}&partitions={w.size}&seed={cfg.seed}"
    g.FromStore(src).ToStore("hbm://fine_in", delete_if_exists=True).SubmitAndWait()
    from dryad_amd.io.providers import provider_for
    g.FromStore("hbm://fine_in").OrderBy(lambda r: r[0:10]).ToStore("hbm://fine_out", delete_if_exists=True) \
        .SubmitAndWait()
    res = g._get_executor().last_result
    assert not {op for _, op, _ in res["fallbacks"]} & {"sample", "separators", "range_partition", "sort"}, \
        res["fallbacks"]
    assert res["exchange"] is not None and "pitch 100" in res["exchange"]["path"], res["exchange"]
    out = provider_for("hbm://fine_out").get("hbm://fine_out")["local"][w.rank].rows
    _valsort(out, w, expect[0], n * w.size)
    kept = provider_for("hbm://fine_in").get("hbm://fine_in")["local"][w.rank].rows   # the input is intact
    assert int(TS.check(kept)[0]) != 0 and kept.shape[0] == n
    base = os.environ.get("FINE_TMP", "/tmp/dryad_fine_rows")
    st = TeraSortStoredJob(cfg, w, f"partfile://{base}/in", f"partfile://{base}/out")
    st.prepare(force=True)
    st.step()
    v = st.validate(*expect)
    assert v["ok"], (w.rank, v)
    assert "pitch 128" in (st.ctx._get_executor().last_result["exchange"] or {}).get("path", ""), \
        st.ctx._get_executor().last_result["exchange"]
    # 3. skew past capacity with the ties kept: the overflowing rank receives into buffers of its
    # own; when HBM cannot hold them, a voted, non-retryable stop within seconds on every rank
    ts = f"gen://terasort?records={200_000 * w.size}&partitions={w.size}&seed=5"
    bufs = RS.SortBuffers.allocate(200_000, 100, w.device, slack=0.01)
    TS.generate(bufs.rows_in[:200_000], w.rank * 200_000, 5)
    bufs.rows_in[:200_000, :10] = 42
    acc_in = TS.check(bufs.rows_in[:200_000]).clone()
    st3 = RS.SortStats()
    out = RS.distributed_sort_rows(bufs, 200_000, 0, 10, w, split_ties=False, stats=st3)
    tot = torch.stack([acc_in[0], TS.check(out)[0], torch.tensor(out.shape[0], device=w.device)])
    shuffle.all_reduce_(tot, "sum", w)
    assert int(tot[0]) == int(tot[1]) and int(tot[2]) == 200_000 * w.size, tot.tolist()
    assert st3.n_out in (0, 200_000 * w.size), st3.n_out          # the one run of equal keys on one rank
    real = RS.SortBuffers.allocate

    def no_hbm(*a, **k):
        raise torch.cuda.OutOfMemoryError("injected: no HBM for a larger receive buffer")
    RS.SortBuffers.allocate = staticmethod(no_hbm)
    TS.generate(bufs.rows_in[:200_000], w.rank * 200_000, 5)
    bufs.rows_in[:200_000, :10] = 42
    t0 = time.perf_counter()
    try:
        RS.distributed_sort_rows(bufs, 200_000, 0, 10, w, split_ties=False)
        raise AssertionError("an overflowing key range without HBM to grow must stop the sort")
    except D.errors.GangAgreementError as e:
        assert not e.retryable and "range partition skew" in str(e), e
    finally:
        RS.SortBuffers.allocate = real
    assert time.perf_counter() - t0 < 10, time.perf_counter() - t0
    # ... and through the query API: OrderBy(k).GroupBy(k) keeps ties (the GroupBy elides its
    # shuffle); bytes 10..13 of every gen://terasort record are equal (00 11 '0' '0'), so one rank
    # receives every row and grows its buffers: one group, oracle-equal
    qctx = D.DryadLinqContext(platform="gpu")
    qctx.PartitionCount = w.size
    k = lambda r: r[10:14]  # noqa: E731
    got = list(qctx.FromStore(ts).OrderBy(k).GroupBy(k, lambda kk, gr: (kk, gr.Count())))
    assert [(bytes(a), c) for a, c in got] == [(b"\x00\x11" + b"00", 200_000 * w.size)], got
    # 4. every key equal with ties split: the E128 path spreads the run over the ranks
    TS.generate(bufs.rows_in[:200_000], w.rank * 200_000, 5)
    bufs.rows_in[:200_000, :10] = 42
    stt = RS.SortStats()
    out = RS.distributed_sort_rows(bufs, 200_000, 0, 10, w, stats=stt)
    assert "E128" in stt.path and abs(stt.n_out - 200_000) <= 2_000, (stt.path, stt.n_out)
    assert torch.equal(out[:, :10], torch.full_like(out[:, :10], 42))
    # 5. a table of 64-byte rows keyed by bytes 8..15 (not the TeraSort layout), OrderBy and
    # OrderByDescending through the query API: the fine-bucket exchange with the key read at its
    # offset (inverted for the descending sort); every rank's output is its exact slice of the
    # stable global order (ties by source rank, then row)
    _rows64(w, base)
    # 6. a COLUMNAR table (gen://records64: 8 int64 columns) by r.V1 (31-bit values) and
    # descending by r.Key (few distinct keys: long runs of ties), packed into byte-keyed rows
    _records64(w)
    w.barrier()
    if w.rank == 0:
        print("FINE_ROWS_OK", w.size, flush=True)
    torch.cuda.synchronize()
    shutdown()


if __name__ == "__main__":
    main()
