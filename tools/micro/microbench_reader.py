"""Page cache -> HBM bandwidth of the chunked pinned reader (io/reader.py) vs the old
read() -> bytearray -> pageable H2D path.  The file is written first (so it sits in the page cache).

    python tools/micro/microbench_reader.py [GB]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    from dryad_amd.io import reader as RD
    d = os.environ.get("TMPDIR", "/tmp")
    p = os.path.join(d, "dryad_reader_bench.bin")
    n = int(gb * 1e9)
    blk = np.random.default_rng(0).integers(0, 256, size=1 << 26, dtype=np.uint8)
    with open(p, "wb") as f:
        left = n
        while left > 0:
            k = min(left, blk.shape[0])
            f.write(blk[:k].tobytes())
            left -= k
    dev = torch.device("cuda")
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    RD.read_to_device(p, dev, out=out)                 # warm: ring registration, page cache
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        RD.read_to_device(p, dev, out=out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ok = torch.equal(out[: blk.shape[0]].cpu(), torch.from_numpy(blk[: min(n, blk.shape[0])]))
    t0 = time.perf_counter()
    with open(p, "rb") as f:
        data = f.read()
    old = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    torch.cuda.synchronize()
    t_old = time.perf_counter() - t0
    del old, data
    os.remove(p)
    best = min(ts)
    print(json.dumps({"bytes": n, "reader_GBps": round(n / best / 1e9, 2), "reader_s": [round(t, 3) for t in ts],
                      "old_path_GBps": round(n / t_old / 1e9, 2), "chunk_MB": RD.CHUNK >> 20, "slots": RD.SLOTS,
                      "threads": RD.THREADS, "verified": bool(ok)}))


if __name__ == "__main__":
    main()
