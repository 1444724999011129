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
region group by group: an order-independent fingerprint of every output group (key, count, sum,
min, max) against the same fingerprint of a reference GroupBy computed by torch sort + scatter ops
over the regenerated input, one key range at a time (dryad_amd/utils/validate.py); plus the
count / V1 totals.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

if "--loopback-ranks" in sys.argv:
    # the loopback harness runs all W sources' stage A in this one process to simulate the
    # exchange; with the default caching allocator that fragments HBM, and one step's stage B in
    # three paid fresh allocations (1.8 s: profiles/r5/gb_lb8_final.log).  Expandable segments
    # keep every step steady (94.3-95.3 ms, profiles/r5/gb_lb8_expandable.log); the per-rank
    # program is unchanged.  Set before torch initialises the device.
    os.environ.setdefault("PYTORCH_HIP_ALLOC_CONF", "expandable_segments:True")

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
    ap.add_argument("--loopback-ranks", type=int, default=0,
                    help="run the per-rank program of a W-rank job on this one GPU (runtime/loopback.py): the "
                         "all-to-all-v replaced by running every other source's stage untimed; reports per-rank ms")
    ap.add_argument("--loopback-rank", type=int, default=0)
    ap.add_argument("--aggregation", choices=("auto", "radix", "sort"), default="auto",
                    help="GroupByAggregation context property (single integer key strategy)")
    ap.add_argument("--hbm-budget-gb", type=float, default=None,
                    help="HbmBudgetBytes: a partition past it is aggregated chunk by chunk (runtime/stream_agg.py), "
                         "e.g. --records-per-gpu 6.25e9 (400 GB) --hbm-budget-gb 60")
    ap.add_argument("--stream-shuffle", action="store_true",
                    help="with --loopback-ranks: the pipelined streamed shuffle (runtime/stream_shuffle.py: rounds "
                         "of chunk partial -> exchange -> fold); per-round times measured, the node step modelled")
    ap.add_argument("--chunk-gb", type=float, default=4.0, help="StreamChunkBytes of --stream-shuffle")
    ap.add_argument("--model-link-GBps", type=float, nargs="*", default=[300.0, 450.0],
                    help="with --loopback-ranks: MODELLED per-rank step with the exchange on a link of this many "
                         "GB/s per GPU (labelled modelled)")
    ap.add_argument("--raw-shuffle", action="store_true",
                    help="with --loopback-ranks: shuffle the pruned raw rows (Select -> HashPartition -> GroupBy) "
                         "instead of partial aggregation before the shuffle")
    ap.add_argument("--source", choices=("gen", "host", "partfile"), default="gen",
                    help="host / partfile: the records are first written (untimed) to a host:// table (pinned "
                         "host columns) or a partfile:// table, and the timed GroupBy reads them from there")
    a = ap.parse_args()
    if a.loopback_ranks:
        return loopback(a)
    w = world()
    import torch
    import dryad_amd as D
    from dryad_amd.io.providers import provider_for
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = w.size
    if a.hbm_budget_gb:
        ctx.HbmBudgetBytes = int(a.hbm_budget_gb * 1e9)
    ctx.GroupByAggregation = a.aggregation
    n = int(a.records_per_gpu) * w.size
    src = f"gen://records64?count={n}&partitions={w.size}&keys={int(a.keys)}&seed=4242" + \
        ("&bounds=0" if a.no_bounds else "")
    out = "hbm://groupby_out"
    if a.source != "gen":                 # the stored input, written once before the timed steps
        stored = "host://groupby_src" if a.source == "host" else "partfile:///tmp/dryad_groupby_src.pt"
        t0 = time.perf_counter()
        ctx.FromStore(src).ToStore(stored, delete_if_exists=True).SubmitAndWait()
        if w.rank == 0:
            print(f"[groupby] wrote {stored} in {time.perf_counter() - t0:.1f}s", flush=True)
        src = stored

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
    valid, fpv = None, None
    if not a.no_validate:
        from dryad_amd.utils import validate as V
        tab = provider_for(out).get(out)["local"]
        cnt = sum(int(t.col(1).sum()) for t in tab.values())
        s1 = sum(int(t.col(2).sum()) for t in tab.values())
        groups = sum(t.n for t in tab.values())
        got_fp = V.combine([V.group_fingerprint([t.col(j) for j in range(5)]) for t in tab.values()])
        del tab
        torch.cuda.empty_cache()
        from dryad_amd.ops import relational as R
        lo = (n * w.rank) // w.size
        hi = (n * (w.rank + 1)) // w.size
        cols = [torch.empty(hi - lo, dtype=torch.int64, device=w.device) for _ in range(2)]
        R.gen_records64(cols, lo, int(a.keys), 4242)
        s_in = int(cols[1].sum())
        del cols
        exp_fp = _expected_groups(n, int(a.keys), w.size, w.rank, w.device)
        i64 = lambda x: x - (1 << 64) if x >= (1 << 63) else x  # noqa: E731
        tot = torch.tensor([cnt, s1, s_in, groups, got_fp[0], i64(got_fp[1]), exp_fp[0], i64(exp_fp[1])],
                           dtype=torch.int64, device=w.device)
        if w.size > 1:
            torch.distributed.all_reduce(tot)
        cnt, s1, s_in, groups, gn, gf, en, ef = tot.tolist()
        fpv = dict(groups=gn, expected_groups=en, fingerprint=gf & ((1 << 64) - 1),
                   expected_fingerprint=ef & ((1 << 64) - 1))
        fpv["ok"] = gn == en and (gf - ef) % (1 << 64) == 0
        valid = cnt == n and s1 == s_in and fpv["ok"]
    med = sorted(times)[len(times) // 2]
    streamed = [v for v in (ex.last_result.get("streamed") or {}).values() if v.get("kind") == "streamed aggregation"]
    report(w, {
        "metric": "GroupBy-Aggregate GB/s of input (10B x 64-byte records at 8 GPUs)",
        "value": round(n * 64 / med / 1e9, 3), "unit": "GB/s", "n_gpus": w.size, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(med * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic gen://records64 (uniform keys)",
        "validated": valid, "groups": groups if valid is not None else None, "host_fallback_ops": fallbacks,
        "validation": None if fpv is None else dict(fpv, method="per-group fingerprint vs a torch sort + scatter "
                                                           "GroupBy of the regenerated input (utils/validate.py)"),
        "all_step_ms": [round(t * 1e3, 2) for t in times],
        "config": {"model": "GroupBy(Key) -> Count/Sum/Min/Max (decomposable, hash shuffle)",
                   "records": n, "record_bytes": 64, "keys": int(a.keys), "parallelism": f"dp{w.size}",
                   "source": {"gen": "gen://records64 generated in the step",
                              "host": "host:// pinned host columns written before the steps (read in the step)",
                              "partfile": "partfile:// table written before the steps (read in the step)"}[a.source],
                   "column_bounds": "measured in the step" if a.no_bounds else (
                       "declared by the generator" if a.source == "gen" else
                       "kept in the stored table's schema" if a.source == "partfile" else "carried by the host table"),
                   "hbm_budget_bytes": ctx.HbmBudgetBytes, "aggregation": a.aggregation,
                   "streamed_aggregation": streamed[0] if streamed else None}})


def loopback(a):
    """Rank ``--loopback-rank`` of a ``--loopback-ranks``-rank GroupBy on one GPU: stage A (read ->
    partial GroupBy -> hash partition) and stage B (final GroupBy) timed, the exchange simulated.
    Validated: every group of this rank's hash range is complete (count and V1 sum of its groups
    against the rank's share of the input, computed by a host-side pass over the same generator)."""
    import json
    import torch
    import dryad_amd as D
    from dryad_amd.compiler.planner import compile_queries
    from dryad_amd.runtime.loopback import LoopbackRank
    W, r = a.loopback_ranks, a.loopback_rank
    n = int(a.records_per_gpu) * W
    src = f"gen://records64?count={n}&partitions={W}&keys={int(a.keys)}&seed=4242" + ("&bounds=0" if a.no_bounds else "")
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = W
    res = lambda k, g: (k, g.Count(), g.Sum(lambda x: x[1]), g.Min(lambda x: x[2]), g.Max(lambda x: x[3]))  # noqa: E731
    q = ctx.FromStore(src)
    if a.raw_shuffle:
        q = q.Select(lambda x: (x[0], x[1], x[2], x[3])).HashPartition(lambda x: x[0], W).GroupBy(lambda x: x[0], res)
    else:
        q = q.GroupBy(lambda x: x[0], res)
    if a.stream_shuffle:
        ctx.StreamShuffle = True
        ctx.StreamChunkBytes = int(a.chunk_gb * 1e9)
        if a.hbm_budget_gb:
            ctx.HbmBudgetBytes = int(a.hbm_budget_gb * 1e9)
    plan = compile_queries(ctx, [q.ToStore("hbm://groupby_lb", delete_if_exists=True)])
    if a.stream_shuffle:
        from dryad_amd.runtime.loopback import LoopbackStreamShuffle
        job = LoopbackStreamShuffle(plan, W, r, ctx)
        job.bytes = {}
    else:
        job = LoopbackRank(plan, W, r)
    ms, ph = [], []
    for i in range(a.warmup + a.steps):
        p = job.step()
        print(f"[groupby-lb] {'warmup' if i < a.warmup else 'step'} {i}: {job.ms:.2f} ms {p} {job.bytes}",
              flush=True)
        if a.stream_shuffle and i >= a.warmup:
            print(f"[groupby-lb] modelled: {[job.model(x) for x in a.model_link_GBps]}", flush=True)
        if i >= a.warmup:
            ms.append(job.ms)
            ph.append(p)
    valid = None
    if not a.no_validate:
        from dryad_amd.utils import validate as V
        out = job.out
        cnt, s1, groups = int(out.col(1).sum()), int(out.col(2).sum()), out.n
        got = V.group_fingerprint([out.col(j) for j in range(5)])
        job.out = out = None
        torch.cuda.empty_cache()
        # the groups of the keys hashed to rank r, from every source partition: the reference
        # GroupBy (torch sort + scatter) of the regenerated rows, one key range at a time
        exp = _expected_groups(n, int(a.keys), W, r, "cuda", keep=lambda k: _dest_of(k, W) == r)
        valid = dict(ok=got == exp, records=cnt, groups=groups, expected_groups=exp[0],
                     fingerprint_match=got[1] == exp[1],
                     method="per-group fingerprint vs a torch sort + scatter GroupBy of the regenerated input")
    mean = sum(ms) / len(ms)
    print(json.dumps({
        "metric": f"GroupBy-Aggregate per-rank step of a {W}-rank job (loopback on one GPU: all-to-all-v replaced)",
        "value": round(mean, 3), "unit": "ms", "higher_is_better": False, "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(mean, 3), "dtype": "int64",
        "data": "synthetic gen://records64 (uniform keys)",
        "config": {"model": "GroupBy(Key) -> Count/Sum/Min/Max", "records_per_rank": int(a.records_per_gpu),
                   "keys": int(a.keys), "ranks": W, "rank": r,
                   "plan": "Select(4 cols) -> HashPartition -> GroupBy (raw rows shuffled)" if a.raw_shuffle else
                   "streamed shuffle: rounds of chunk partial -> HashPartition -> exchange -> fold (pipelined)"
                   if a.stream_shuffle else "partial GroupBy -> HashPartition -> final GroupBy",
                   "phases_ms": {k: round(sum(p[k] for p in ph) / len(ph), 3) for k in ph[0]},
                   "exchange": {k: v for k, v in job.bytes.items()},
                   # the exchange is not run here: MODELLED node steps from the measured compute and an
                   # assumed per-GPU link rate
                   "modelled_exchange": ([job.model(x) for x in a.model_link_GBps] if a.stream_shuffle else
                                         [_bulk_model(job, x) for x in a.model_link_GBps]),
                   "stream": getattr(job, "stats", None),
                   "per_rank_input_GBps": round(int(a.records_per_gpu) * 64 / 1e6 / mean, 1),
                   "validated": valid}}), flush=True)


def _bulk_model(job, link):
    from dryad_amd.runtime.loopback import bulk_model
    return bulk_model(job.phases, job.bytes, link)


def _gen_chunks(n: int, keys: int, step: int = 1 << 27):
    """Callable -> iterator over [Key, V1, V2, V3] int64 chunks of gen://records64 rows 0..n-1."""
    import torch
    from dryad_amd.ops import relational as R

    def it():
        for c0 in range(0, n, step):
            c1 = min(n, c0 + step)
            cols = [torch.empty(c1 - c0, dtype=torch.int64, device="cuda") for _ in range(4)]
            R.gen_records64(cols, c0, keys, 4242)
            yield cols
    return it


def _expected_groups(n: int, keys: int, W: int, rank: int, dev, keep=None):
    """(groups, fingerprint) of the reference GroupBy over this rank's share of the key ranges (every
    rank regenerates all n rows per range; ``keep`` selects rows of the groups it validates)."""
    from dryad_amd.utils import validate as V
    pieces = max(16, 8 * W) if keep is None else 16
    ranges = V.key_ranges(0, keys - 1, pieces)
    mine = ranges if keep is not None else [r for i, r in enumerate(ranges) if i % W == rank]
    return V.expected_fingerprint(_gen_chunks(n, keys), ["count", "sum", "min", "max"], mine, keep=keep)


def _dest_of(keys, W):
    """Destination rank of int64 keys under the executor's hash partition (gpu/ops.op_hash_partition)."""
    from dryad_amd.ops import relational as R
    from dryad_amd.gpu import ops as G
    from dryad_amd.gpu.table import DeviceTable, Shape
    t = DeviceTable.from_columns({"k": keys}, Shape("scalar", ["k"]))
    k, tup = G.hash_keys(t, lambda x: x)
    e, _ = R.stable_hash_dest(k, t.n, W, tup, keys.device, ports=False)
    return e[:, 1] if e.dim() == 2 else e


if __name__ == "__main__":
    main()
