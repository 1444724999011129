"""PCIe host <-> HBM throughput, one direction and both at once, by the DMA engines
(hipMemcpyAsync in 512 MB pieces, as ops/extsort._copy issues them) and by a CU copy kernel that
reads or writes the page-locked host buffer through its device mapping (ops/channel.copy_wide).

    python tools/micro/microbench_pcie.py [GB per direction] [--grids 256,1024]

The out-of-core sort's bucket phase streams one direction up and the other down at the same
time; this measures which engine mix moves the most bytes per second.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import _lib  # noqa: E402
from dryad_amd.ops import channel as CH  # noqa: E402

PIECE = 512 << 20


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 8.0
    grids = [0]
    if "--grids" in sys.argv:
        grids = [int(x) for x in sys.argv[sys.argv.index("--grids") + 1].split(",")]
    n = int(gb * 1e9) // PIECE * PIECE
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    host_up = _lib.PinnedHostBuffer((n,))
    host_dn = _lib.PinnedHostBuffer((n,))
    host_up.tensor.fill_(7)
    print(f"pinned 2 x {n / 1e9:.1f} GB in {time.perf_counter() - t0:.1f}s", flush=True)
    d_up = torch.empty(n, dtype=torch.uint8, device=dev)
    d_dn = torch.full((n,), 3, dtype=torch.uint8, device=dev)
    s_up, s_dn = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def dma_up():
        for a in range(0, n, PIECE):
            _lib.memcpy_async(d_up[a:a + PIECE], host_up.tensor[a:a + PIECE], s_up)

    def dma_dn():
        for a in range(0, n, PIECE):
            _lib.memcpy_async(host_dn.tensor[a:a + PIECE], d_dn[a:a + PIECE], s_dn)

    def k_up(grid):
        return lambda: CH.copy_wide(d_up, host_up.tensor, s_up, grid)

    def k_dn(grid):
        return lambda: CH.copy_wide(host_dn.tensor, d_dn, s_dn, grid)

    def run(name, fns, reps=3):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for f in fns:
                f()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        moved = n * len(fns)
        print(f"{name:40s} {best * 1e3:8.1f} ms  {moved / best / 1e9:6.1f} GB/s total "
              f"({n / best / 1e9:5.1f} per direction)", flush=True)

    run("dma up", [dma_up])
    run("dma down", [dma_dn])
    run("dma up + dma down", [dma_up, dma_dn])
    for g in grids:
        run(f"kernel up (grid {g or 'auto'})", [k_up(g)])
        run(f"kernel down (grid {g or 'auto'})", [k_dn(g)])
        run(f"dma up + kernel down (grid {g or 'auto'})", [dma_up, k_dn(g)])
        run(f"kernel up + dma down (grid {g or 'auto'})", [k_up(g), dma_dn])
        run(f"kernel up + kernel down (grid {g or 'auto'})", [k_up(g), k_dn(g)])
    ok_up = bool(torch.equal(d_up[:PIECE].cpu(), host_up.tensor[:PIECE]))
    ok_dn = bool(torch.equal(host_dn.tensor[-PIECE:], d_dn[-PIECE:].cpu()))
    print(f"copies correct: up={ok_up} down={ok_dn}", flush=True)


if __name__ == "__main__":
    main()
