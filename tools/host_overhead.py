"""Host time of one TeraSort query job on the GPU executor with a tiny input (the device work is
negligible, so the wall time is the per-job Python / runtime overhead that the headline bench pays
between steps), with a cProfile of the job thread.

    python tools/host_overhead.py [records] [steps]
"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dryad_amd as D  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = 1
    src = f"gen://terasort?records={n}&partitions=1&seed=1"

    def step():
        q = ctx.FromStore(src).OrderBy(lambda r: r[0:10]).ToStore("hbm://terasort_out", delete_if_exists=True)
        ctx._freeze()
        ctx._get_executor().run_job([q], None)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"records={n}: {1e3 * (time.perf_counter() - t) / steps:.3f} ms per job")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(40)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    main()
