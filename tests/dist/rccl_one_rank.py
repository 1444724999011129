"""The multi-rank exchange code against REAL RCCL on a one-GPU box: a one-rank RCCL communicator
(torch.distributed backend "nccl") and a World with ``force_collectives``, so every data movement
that a W-rank job makes through the process group is made here too, with W = 1 (run by
tests/test_gpu_multirank.py).  RCCL refuses two ranks on one device ("Duplicate GPU detected",
profiles/r4/nccl_two_ranks_one_gpu_probe.log), so this is the one way a single-GPU box runs the
RCCL branches of parallel/shuffle.py and ops/recordsort.py:

  * the shuffle primitives: count exchange, all-to-all-v (one collective and the chunked P2P
    rounds), the asynchronous all-to-all-v handle, gang status, all-gathers, all-reduce, broadcast;
  * the fine-bucket OrderBy over a materialised table (sampler all-gather, fine counts all-to-all,
    gang agreements, voted capacity check, B asynchronous payload rounds, tile merge), validated;
  * the E128 range-partition path (OrderByDescending), validated.
"""
import datetime
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402
from dryad_amd.parallel import shuffle  # noqa: E402
from dryad_amd.parallel.comm import World  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29657")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=120), device_id=dev)
    w = World(rank=0, size=1, local_rank=0, device=dev, backend="nccl", force_collectives=True)
    try:
        # 1. primitives
        x = torch.randint(0, 256, (3 << 20,), dtype=torch.uint8, device=dev)
        r = torch.empty_like(x)
        shuffle.alltoallv_bytes(x, [x.numel()], r, [x.numel()], w)
        assert torch.equal(r, x)
        r.zero_()
        h = shuffle.alltoallv_bytes_async(x, [x.numel()], r, [x.numel()], w)
        assert h is not None, "RCCL all-to-all-v should be asynchronous"
        shuffle.wait(h)
        torch.cuda.synchronize()
        assert torch.equal(r, x)
        keep = shuffle.CHUNK_BYTES
        shuffle.CHUNK_BYTES = 1 << 20               # the chunked P2P rounds
        try:
            r.zero_()
            shuffle.alltoallv_bytes(x, [x.numel()], r, [x.numel()], w)
            assert torch.equal(r, x)
        finally:
            shuffle.CHUNK_BYTES = keep
        assert shuffle.exchange_counts(torch.tensor([12345]), w).tolist() == [12345]
        assert shuffle.gang_status(True, 7, w) == [(True, 7)]
        v = torch.arange(10, dtype=torch.int64, device=dev).view(5, 2)
        assert torch.equal(shuffle.all_gather_varlen(v, w), v)
        t = torch.tensor([3.0], device=dev)
        assert float(shuffle.all_reduce_(t, "max", w)) == 3.0
        assert float(shuffle.broadcast_(t, 0, w)) == 3.0
        # 2. the fine-bucket OrderBy over a table read in place
        n = int(os.environ.get("TS_RECORDS", "3000000"))
        src = torch.empty((n, 100), dtype=torch.uint8, device=dev)
        TS.generate(src, 0, 4242)
        acc_in = TS.check(src).clone()
        bufs = RS.SortBuffers.allocate(int(n * 1.01) + 1024, 100, dev)
        st = RS.SortStats()
        RS.PIPE_SUBS = 4
        out = RS.distributed_sort_rows(bufs, n, 0, 10, w, stats=st, src=src)
        acc = TS.check(out)
        torch.cuda.synchronize()
        assert st.path.startswith("fine-bucket exchange over the table"), st.path
        assert out.shape[0] == n and int(acc[1]) == 0 and int(acc[0]) == int(acc_in[0]), (acc.tolist(), acc_in.tolist())
        rep = st.exchange_report()
        assert rep["rounds"] == 4 and "round_arrival_ms" in rep, rep
        # the send side overlapped with the exchange: each round packed just before it went out,
        # received into slots, merged from there
        assert "rounds packed as they go out" in st.path and "first_round_queued_ms" in rep, rep
        assert rep["overlap"]["slots"] == RS.OVERLAP_SLOTS and not rep["overlap"]["skew_fixups"], rep
        # 3. descending: the fine-bucket exchange with inverted key windows
        st2 = RS.SortStats()
        out2 = RS.distributed_sort_rows(bufs, n, 0, 10, w, stats=st2, src=src, descending=True)
        asc = out2.flip(0).contiguous()
        acc2 = TS.check(asc)
        torch.cuda.synchronize()
        assert st2.path.startswith("fine-bucket exchange over the table"), st2.path
        assert out2.shape[0] == n and int(acc2[1]) == 0 and int(acc2[0]) == int(acc_in[0]), acc2.tolist()
        # 3b. a 12-byte key (past the fine path's 10): the E128 range-partition path
        st3 = RS.SortStats()
        out3 = RS.distributed_sort_rows(bufs, n, 0, 12, w, stats=st3, src=src)
        acc3 = TS.check(out3)
        torch.cuda.synchronize()
        assert st3.path.startswith("E128"), st3.path
        assert out3.shape[0] == n and int(acc3[1]) == 0 and int(acc3[0]) == int(acc_in[0]), acc3.tolist()
        del bufs, src, out, out2, out3
        torch.cuda.empty_cache()
        # 4. the bench's N > 1 program: the DryadLINQ query through the executor's fused OrderBy gang
        #    stage (ExchangeOneRank plans the sampled range shuffle for the one partition), validated
        from dryad_amd.models.terasort import TeraSortConfig, TeraSortQueryJob
        from dryad_amd.parallel.comm import set_world
        set_world(w)
        job = TeraSortQueryJob(TeraSortConfig(records_per_rank=n), w)
        expect = job.input_checksum()
        job.step()
        val = job.validate(*expect)
        q = job.executor_report()
        assert val["ok"], val
        assert q["exchange"] and q["exchange"]["path"].startswith("fine-bucket exchange over the table"), q
        assert not q["fallbacks"], q
        print(f"RCCL_ONE_RANK_OK fine={rep['round_arrival_ms']} desc={st2.path} query={q['exchange']['path']}",
              flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
