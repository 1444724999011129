"""Device record codec throughput on a 10 GB part (HBM -> HBM; no I/O):

    python tools/micro/codec_bw.py [GB]

* fixed-width records (8 x Int64 = 64 bytes): decode (rows -> columns) and encode;
* variable-length records (Int64 key, a 12..40-character string, a Float64): record-boundary
  discovery without a sidecar (device speculative chains, csrc/kernels/varscan.hip, vs the host
  scan) and decode with the found block index.
GB/s = part bytes / kernel time (best of 3, HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dryad_amd import types as T  # noqa: E402
from dryad_amd.ops import codec as CD  # noqa: E402


def timed(fn, reps=3):
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = e0.elapsed_time(e1) if best is None else min(best, e0.elapsed_time(e1))
    return best


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    dt = T.RecordT([(f"f{i}", T.Int64) for i in range(8)], tuple)
    n = int(gb * 1e9) // 64
    buf = torch.randint(0, 256, (n * 64,), dtype=torch.uint8, device="cuda")
    t = CD.decode(buf, dt)
    ms = timed(lambda: CD.decode(buf, dt))
    print(f"fixed decode: {n * 64 / 1e9:.1f} GB in {ms:.2f} ms = {n * 64 / 1e6 / ms:.0f} GB/s", flush=True)
    ms = timed(lambda: CD.encode(t, dt))
    print(f"fixed encode: {n * 64 / 1e9:.1f} GB in {ms:.2f} ms = {n * 64 / 1e6 / ms:.0f} GB/s", flush=True)
    assert torch.equal(CD.encode(t, dt), buf)
    del t, buf
    # variable-length: records of an Int64, a string and a Float64, built on the host once and tiled
    from dryad_amd.io import binary as B
    vdt = T.RecordT([("k", T.Int64), ("s", T.String), ("x", T.Float64)], tuple)
    rng = np.random.default_rng(1)
    alpha = "abcdefghijklmnopqrstuvwxyz"
    recs = [(i, "".join(alpha[j] for j in rng.integers(0, 26, size=int(rng.integers(12, 41)))), i * 0.5)
            for i in range(200_000)]
    blob = B.encode_records(vdt, recs)
    reps = max(1, int(gb * 1e9) // len(blob))
    part = np.tile(np.frombuffer(blob, dtype=np.uint8), reps)
    import time
    t0 = time.time()
    n_idx, offs = CD.block_index_host(part, vdt)
    th = time.time() - t0
    dbuf = torch.from_numpy(part).cuda()
    got = CD.block_index_device(dbuf, vdt)
    assert got is not None and got[0] == n_idx and torch.equal(got[1].cpu(), torch.from_numpy(offs)), "boundary mismatch"
    ms = timed(lambda: CD.block_index_device(dbuf, vdt))
    print(f"string boundaries (device, no sidecar): {part.size / 1e9:.1f} GB in {ms:.2f} ms = "
          f"{part.size / 1e6 / ms:.0f} GB/s (host scan {th * 1e3:.0f} ms = {part.size / 1e9 / th:.1f} GB/s) "
          f"{CD.LAST_SCAN}", flush=True)
    doffs = got[1]
    ms = timed(lambda: CD.decode_var(dbuf, vdt, n_idx, doffs))
    print(f"string decode: {part.size / 1e9:.1f} GB ({n_idx} records) in {ms:.2f} ms = {part.size / 1e6 / ms:.0f} GB/s",
          flush=True)


if __name__ == "__main__":
    main()
