"""Allocation-order A/B for the plain (100-byte pitch) sort buffer set of the direct TeraSort path
(the layout the multi-rank sort uses): rows_in before rows_out (as allocated) or swapped.  Run once
per order, each in a fresh process:

    python tools/ab_alloc_order_direct.py [in-first|out-first] [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dryad_amd.models.terasort import TeraSortConfig, TeraSortJob, run_steps  # noqa: E402
from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402


def out_first(capacity, stride, device, slack=0.0):
    cap = int(capacity * (1.0 + slack)) + 1024
    rows_out = torch.empty((cap, stride), dtype=torch.uint8, device=device)
    rows_in = torch.empty((cap, stride), dtype=torch.uint8, device=device)
    return RS.SortBuffers(rows_in=rows_in, rows_out=rows_out,
                          ent_a=torch.empty((cap, 2), dtype=torch.int64, device=device),
                          ent_b=torch.empty((cap, 2), dtype=torch.int64, device=device))


def main():
    order = sys.argv[1] if len(sys.argv) > 1 else "in-first"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    if order == "out-first":
        RS.SortBuffers.allocate = staticmethod(out_first)
    world = init_world(device="cuda")
    job = TeraSortJob(TeraSortConfig(records_per_rank=1_250_000_000), world)
    expect = job.input_checksum()
    torch.cuda.empty_cache()
    for _ in range(3):
        job.step()
    secs = run_steps(job, steps)
    ok = job.validate(*expect)["ok"]
    print(f"{order}: {1e3 * secs / steps:.2f} ms/step validated={ok}", flush=True)


if __name__ == "__main__":
    main()
