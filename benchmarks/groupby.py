"""GroupBy-Aggregate benchmark: GB/s of input aggregated, 10B x 64-byte records at 8 GPUs
(BASELINE.json config "GroupBy-Aggregate 10B x 64-byte records, hash all-to-all over xGMI").

Weak scaling: 1.25e9 records (80 GB) per GPU, 8 GPUs = 10e9 records.  Keys are uniform over
``--keys`` values (default 2^30, so partial aggregation barely shrinks the data and the hash
shuffle moves most of it).  The timed step is one DryadLINQ job through the GPU executor:

    FromStore(gen://records64).GroupBy(r => r.Key,
        (k, g) => (k, g.Count(), g.Sum(r => r.V1), g.Min(r => r.V2), g.Max(r => r.V3)))
      .ToStore(hbm://groupby_out)

i.e. generate (the "read" of the input) -> partial GroupBy (radix sort + segmented reduce) ->
hash partition -> RCCL all-to-all-v -> final GroupBy -> HBM table.  Validated outside the timed
region (group counts and V1 sums against column totals).
"""
from __future__ import annotations

import argparse

from common import report, timed, world  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records-per-gpu", type=float, default=1.25e9)
    ap.add_argument("--keys", type=float, default=float(1 << 30))
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--no-bounds", action="store_true",
                    help="withhold the generator's column bounds (as for a stored table): the dense "
                         "GroupBy path then measures the key range itself, inside the timed step")
    a = ap.parse_args()
    w = world()
    import torch
    import dryad_amd as D
    from dryad_amd.io.providers import provider_for
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = w.size
    n = int(a.records_per_gpu) * w.size
    src = f"gen://records64?count={n}&partitions={w.size}&keys={int(a.keys)}&seed=4242" + \
        ("&bounds=0" if a.no_bounds else "")
    out = "hbm://groupby_out"

    def step():
        q = ctx.FromStore(src).GroupBy(
            lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Min(lambda r: r[2]),
                                          g.Max(lambda r: r[3])))
        q.ToStore(out, delete_if_exists=True).SubmitAndWait()

    for _ in range(a.warmup):
        step()
    times = []
    for _ in range(a.steps):
        dt, _ = timed(w, step)
        times.append(dt)
    ex = ctx._get_executor()
    fallbacks = [f"{s}:{op}" for s, op, _ in ex.last_result.get("fallbacks", [])]
    valid = None
    if not a.no_validate:
        tab = provider_for(out).get(out)["local"]
        cnt = sum(int(t.col(1).sum()) for t in tab.values())
        s1 = sum(int(t.col(2).sum()) for t in tab.values())
        groups = sum(t.n for t in tab.values())
        from dryad_amd.ops import relational as R
        lo = (n * w.rank) // w.size
        hi = (n * (w.rank + 1)) // w.size
        cols = [torch.empty(hi - lo, dtype=torch.int64, device=w.device) for _ in range(2)]
        R.gen_records64(cols, lo, int(a.keys), 4242)
        tot = torch.tensor([cnt, s1, int(cols[1].sum()), groups], dtype=torch.int64, device=w.device)
        if w.size > 1:
            torch.distributed.all_reduce(tot)
        cnt, s1, s_in, groups = tot.tolist()
        valid = cnt == n and s1 == s_in
    med = sorted(times)[len(times) // 2]
    report(w, {
        "metric": "GroupBy-Aggregate GB/s of input (10B x 64-byte records at 8 GPUs)",
        "value": round(n * 64 / med / 1e9, 3), "unit": "GB/s", "n_gpus": w.size, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(med * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic gen://records64 (uniform keys)",
        "validated": valid, "groups": groups if valid is not None else None, "host_fallback_ops": fallbacks,
        "all_step_ms": [round(t * 1e3, 2) for t in times],
        "config": {"model": "GroupBy(Key) -> Count/Sum/Min/Max (decomposable, hash shuffle)",
                   "records": n, "record_bytes": 64, "keys": int(a.keys), "parallelism": f"dp{w.size}",
                   "column_bounds": "measured in the step" if a.no_bounds else "declared by the generator"}})


if __name__ == "__main__":
    main()
