"""Hash-join benchmark: GB/s of input joined, two 100 GB tables of 64-byte rows
(BASELINE.json config "Hash-join two 100 GB tables, spill HBM -> host DRAM").

Strong scaling: the two 100 GB tables are split over the N GPUs (1 GPU: 200 GB of input with
the grace partitions spilled to pinned host DRAM; 8 GPUs: 25 GB per GPU, buckets stay in HBM).
The timed step is the whole join: input generation, grace partitioning (+ xGMI exchange, + host
spill), per-bucket sort-merge joins and the reduction.  Validated against the answer computed
from the probe table alone.
"""
from __future__ import annotations

import argparse

from common import report, timed, world  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table-gb", type=float, default=100.0)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--chunk-rows", type=float, default=float(1 << 27))
    ap.add_argument("--hbm-budget-gb", type=float, default=None)
    ap.add_argument("--no-validate", action="store_true")
    a = ap.parse_args()
    w = world()
    from dryad_amd.models.hashjoin import HashJoinConfig, HashJoinJob
    rows = int(a.table_gb * 1e9 / 64)
    cfg = HashJoinConfig(rows_r=rows, rows_s=rows, chunk_rows=int(a.chunk_rows),
                         hbm_budget=None if a.hbm_budget_gb is None else int(a.hbm_budget_gb * 1e9))
    job = HashJoinJob(w, cfg)
    for _ in range(a.warmup):
        job.step()
    times, res = [], None
    for _ in range(a.steps):
        dt, res = timed(w, job.step)
        times.append(dt)
    ok = None
    if not a.no_validate:
        ok = res == job.expected()
    med = sorted(times)[len(times) // 2]
    total = 2 * rows * 64
    report(w, {
        "metric": "Hash-join GB/s of input (two 100 GB tables, spill HBM -> host DRAM)",
        "value": round(total / med / 1e9, 3), "unit": "GB/s", "n_gpus": w.size, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(med * 1e3, 2), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic gen://records64 row tables (dimension x fact)",
        "validated": ok, "matches": res[0] if res else None, "all_step_ms": [round(t * 1e3, 1) for t in times],
        "spilled_bytes_per_rank": job.last.get("spilled_bytes"), "buckets": job.last.get("buckets"),
        "partition_s": round(job.last.get("partition_s", 0), 3),
        "config": {"model": "R.Join(S, Key).Select(r.V1 + s.V1).Sum() (grace hash join)", "rows_per_table": rows,
                   "row_bytes": 64, "parallelism": f"dp{w.size}"}})


if __name__ == "__main__":
    main()
