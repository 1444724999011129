"""Per-op HBM peak of the multi-rank shuffle memcheck (tests/dist/gpu_query_sweep_ranks.py):
prints torch.cuda.max_memory_allocated() after every operator of every stage."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dryad_amd as D  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402
from dryad_amd.runtime import gpu_executor as GE  # noqa: E402


def main():
    w = init_world(device="cuda")
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = w.size
    n = 2_000_000
    orig_op, orig_gather = GE.GpuJobRunner._run_op, GE.GpuJobRunner._gather_inputs

    def run_op(self, *a, **k):
        out = orig_op(self, *a, **k)
        s = a[3] if len(a) > 3 else k["s"]
        op = a[0]
        torch.cuda.synchronize()
        if w.rank == 0:
            print(f"[mem] {s.name}:{op['op']}: alloc {torch.cuda.memory_allocated() / 1e6:.1f} MB, "
                  f"peak {torch.cuda.max_memory_allocated() / 1e6:.1f} MB", flush=True)
        return out

    def gather(self, s, *a, **k):
        out = orig_gather(self, s, *a, **k)
        torch.cuda.synchronize()
        if w.rank == 0:
            print(f"[mem] {s.name}:gather: alloc {torch.cuda.memory_allocated() / 1e6:.1f} MB, "
                  f"peak {torch.cuda.max_memory_allocated() / 1e6:.1f} MB", flush=True)
        return out
    GE.GpuJobRunner._run_op, GE.GpuJobRunner._gather_inputs = run_op, gather
    for _ in range(2):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        print(f"[mem] base {torch.cuda.memory_allocated() / 1e6:.1f} MB (partition {n * 64 / 1e6:.1f} MB)", flush=True)
        g.FromStore(f"gen://records64?count={n * w.size}&partitions={w.size}&keys=1000000&seed=3").HashPartition(
            lambda r: r[0], w.size).ToStore("hbm://memprobe", delete_if_exists=True).SubmitAndWait()


if __name__ == "__main__":
    main()
