"""parallel/shuffle.py's all-to-all-v on N gloo CPU ranks with a tiny chunk size, so every pair
above DRYAD_SHUFFLE_CHUNK_BYTES goes through the chunked batch_isend_irecv rounds (the branch a
125 GB per GPU shuffle takes over RCCL): uneven counts (zeros, below, at and far above the chunk),
payload bytes checked against what every source rank generated for this rank."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.parallel import shuffle  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402

CHUNK = 1000


def count(src, dst, case):
    return [0, 7, CHUNK, CHUNK + 1, 5 * CHUNK + 17][(src * 3 + dst * 5 + case) % 5]


def payload(src, dst, n):
    return ((torch.arange(n, dtype=torch.int64) * 31 + src * 101 + dst * 7) % 251).to(torch.uint8)


def main():
    w = init_world(device="cpu")
    W, me = w.size, w.rank
    shuffle.CHUNK_BYTES = CHUNK
    for case in range(3):
        sc = [count(me, d, case) for d in range(W)]
        rc = [count(s, me, case) for s in range(W)]
        send = torch.cat([payload(me, d, sc[d]) for d in range(W)] + [torch.zeros(3, dtype=torch.uint8)])
        recv = torch.full((sum(rc) + 5,), 0xEE, dtype=torch.uint8)
        got_counts = shuffle.exchange_counts(torch.tensor(sc, dtype=torch.int64), w).tolist()
        assert got_counts == rc, (me, got_counts, rc)
        if case == 2:
            shuffle.wait(shuffle.alltoallv_bytes_async(send, sc, recv, rc, w))
        else:
            shuffle.alltoallv_bytes(send, sc, recv, rc, w)
        off = 0
        for s in range(W):
            assert torch.equal(recv[off: off + rc[s]], payload(s, me, rc[s])), (me, s, case)
            off += rc[s]
        assert torch.equal(recv[off:], torch.full((5,), 0xEE, dtype=torch.uint8)), "wrote past the receive counts"
    # the branch an RCCL run takes below the chunk size: tensors where the backend moves them (host
    # memory under gloo, HBM under RCCL) -> one asynchronous all_to_all_single with split sizes,
    # a real work handle that the caller waits for later (recordsort's pipelined rounds)
    shuffle.CHUNK_BYTES = 1 << 30
    for case in range(2):
        sc = [count(me, d, case) for d in range(W)]
        rc = [count(s, me, case) for s in range(W)]
        send = torch.cat([payload(me, d, sc[d]) for d in range(W)])
        recv = torch.full((sum(rc),), 0xEE, dtype=torch.uint8)
        h = shuffle.alltoallv_bytes_async(send, sc, recv, rc, w)
        assert (h is not None) == (W > 1), h
        shuffle.wait(h)
        off = 0
        for s in range(W):
            assert torch.equal(recv[off: off + rc[s]], payload(s, me, rc[s])), (me, s, "async", case)
            off += rc[s]
    # the gang agreement before a payload collective: a rank past its capacity stops every rank
    from dryad_amd.errors import GangAgreementError
    from dryad_amd.ops import recordsort as RS
    st = shuffle.gang_status(me != W - 1, me * 10, w)
    assert st == [(r != W - 1, r * 10) for r in range(W)], st
    try:
        RS._check_capacity(100 if me == W - 1 else 10, 50, w)
        raise AssertionError("the over-capacity rank must stop every rank")
    except GangAgreementError as e:
        assert not e.retryable and e.ranks == (W - 1,) and f"rank {W - 1} receives 50 rows past" in str(e), e
    try:
        RS._agree(RuntimeError("boom") if me == 0 else None, w, "test stage")
        raise AssertionError("a failed rank must stop every rank")
    except GangAgreementError as e:
        assert e.retryable and e.ranks == (0,), e
        assert ("boom" in str(e)) == (me == 0), e
    assert RS._agree(None, w, "ok", value=me + 1) == list(range(1, W + 1))
    w.barrier()
    if me == 0:
        print(f"CHUNKED_OK {W}", flush=True)


if __name__ == "__main__":
    main()
    # tear the process group down before the interpreter exits: gloo's threads torn down during
    # finalisation abort the process now and then ("terminate called without an active exception")
    from dryad_amd.parallel.comm import shutdown
    shutdown()
