"""k-means benchmark: seconds per iteration on 1e9 x 128-dim float32 points at 8 GPUs
(BASELINE.json config "k-means on 1B x 128-dim points (Apply/Fork iterative DAG, MFMA reductions)").

Weak scaling like the TeraSort bench: 125M points (64 GB) per GPU, so 8 GPUs hold the named 1B
points.  Every timed iteration is a full DryadLINQ job through the GPU executor: the per-partition
@device_function (fused MFMA assignment + partial sums) over the HBM-resident point table, the
gather of the K partial rows and the combine.  Points are generated once (gen://points ->
hbm://) before timing.

    python benchmarks/kmeans.py [--points-per-gpu 125e6] [--k 64] [--iters 5] [--warmup 1]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 benchmarks/kmeans.py
"""
from __future__ import annotations

import argparse

from common import report, timed, world  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points-per-gpu", type=float, default=125e6)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--blobs", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    w = world()
    import numpy as np
    import dryad_amd as D
    from dryad_amd.models.kmeans import KMeansConfig, KMeansJob
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = w.size
    cfg = KMeansConfig(points_per_partition=int(a.points_per_gpu), k=a.k, blobs=a.blobs)
    t_gen, job = timed(w, lambda: KMeansJob(ctx, cfg, partitions=w.size))
    cents = job.initial_centroids()
    for _ in range(a.warmup):
        cents = job.iterate(cents)
    times = []
    for _ in range(a.iters):
        dt, cents = timed(w, lambda c=cents: job.iterate(c))
        times.append(dt)
    n = job.n
    s_it = float(np.median(times))
    report(w, {
        "metric": "k-means seconds per iteration (1B x 128-dim points at 8 GPUs)", "value": round(s_it, 4),
        "unit": "s/iteration", "n_gpus": w.size, "steps": a.iters, "warmup": a.warmup,
        "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic blob points (gen://points, counter-based), materialised in HBM",
        "points_per_sec": round(n / s_it), "all_iteration_s": [round(t, 4) for t in times],
        "generate_s": round(t_gen, 3),
        "config": {"model": "k-means (DoWhile/ApplyPerPartition/Apply job per iteration)", "points": n,
                   "dim": 128, "k": a.k, "parallelism": f"dp{w.size}"}})


if __name__ == "__main__":
    main()
