"""Hash-join benchmark: GB/s of input joined, two 100 GB tables of 64-byte rows
(BASELINE.json config "Hash-join two 100 GB tables, spill HBM -> host DRAM").

The query goes through the DryadLINQ API:

    R.Join(S, r => r.Key, s => s.Key, (r, s) => r.V1 + s.V1).Sum()

R is a dimension table (keys a bijection of [0, |R|)), S a fact table (keys uniform in [0, |R|)),
both ``gen://records64`` stores.  The GPU executor plans it as the fused grace / radix join stage
(dryad_amd/runtime/fused_join.py): column pruning derived from the traced selectors (Key + V1 of
each side), hash routing over xGMI, HBM-resident buckets up to ``--hbm-budget-gb`` with the rest
spilled to pinned host DRAM, the Sum fused into the probe.  Strong scaling: the two 100 GB tables
are split over the N GPUs.  The timed step is one whole job (planning, input generation = the
read, partitioning, spill, bucket joins, final aggregate).  Validated against the answer computed
independently from S alone (models/hashjoin.HashJoinJob.expected).  ``--direct`` times the
hand-assembled pipeline (models/hashjoin.py) instead, for comparison.
"""
from __future__ import annotations

import argparse

from common import report, timed, world  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table-gb", type=float, default=100.0)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--hbm-budget-gb", type=float, default=None)
    ap.add_argument("--direct", action="store_true")
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--to-store", default=None,
                    help="partfile:// output: time R.Join(S, ..., (r, s) => (r.Key, r.V1, s.V1)).ToStore(uri) instead "
                         "of the Sum (the general grace join stage, pairs streamed bucket by bucket to the part files)")
    ap.add_argument("--names", action="store_true",
                    help="string keys: both tables are gen://names (Name = \"u\" + decimal(Key), V1, V2 from the same "
                         "generator), joined on Name; with --to-store the result is (r.V2, r.V1, s.V1), so the "
                         "validation of the integer-key join applies unchanged")
    ap.add_argument("--name-len", type=int, default=0,
                    help="with --names: every Name padded to this many bytes (> 20; e.g. 200: longer than "
                         "GraceJoinStringBytes, so the join widens its string slots or moves them out of line)")
    ap.add_argument("--string-bytes", type=int, default=24,
                    help="GraceJoinStringBytes: inline bytes per string field in the packed bucket rows")
    a = ap.parse_args()
    w = world()
    import dryad_amd as D
    from dryad_amd.models.hashjoin import SEED_R, SEED_S, HashJoinConfig, HashJoinJob
    rows = int(a.table_gb * 1e9 / 64)
    budget = None if a.hbm_budget_gb is None else int(a.hbm_budget_gb * 1e9)
    cfg = HashJoinConfig(rows_r=rows, rows_s=rows, hbm_budget=budget)
    job = HashJoinJob(w, cfg) if a.direct else None
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = w.size
    if budget is not None:
        ctx.HbmBudgetBytes = budget
    if a.to_store:
        ctx.PartFileSplitBytes = 1 << 30      # a rank's output partition over 8 part files at once
    gen = "names" if a.names else "records64"
    nl = f"&namelen={a.name_len}" if a.names and a.name_len else ""
    R = f"gen://{gen}?count={rows}&partitions={w.size}&keys={rows}&seed={SEED_R}&mode=dim{nl}"
    S = f"gen://{gen}?count={rows}&partitions={w.size}&keys={rows}&seed={SEED_S}{nl}"
    if a.names:
        ctx.GraceJoin = True
        ctx.GraceJoinStringBytes = a.string_bytes

    def api_step():
        total = ctx.FromStore(R).Join(ctx.FromStore(S), lambda r: r[0], lambda s: s[0],
                                      lambda r, s: r[1] + s[1]).Sum()
        return [ctx._get_executor().last_result["join"]["matches"], total]

    def store_step():
        sel = (lambda r, s: (r[2], r[1], s[1])) if a.names else (lambda r, s: (r[0], r[1], s[1]))
        ctx.FromStore(R).Join(ctx.FromStore(S), lambda r: r[0], lambda s: s[0], sel) \
            .ToStore(a.to_store, delete_if_exists=True).SubmitAndWait()
        return None

    def store_check():
        """(pairs, sum of r.V1 + s.V1, pair fingerprint) over the written part files, streamed back
        through HBM (the fingerprint: utils/validate.group_fingerprint of every output record)."""
        import torch
        from dryad_amd.io import partfile as PF
        from dryad_amd.io import reader as RD
        from dryad_amd.io.providers import parse_uri
        from dryad_amd.utils import validate as V
        meta = PF.read_meta(parse_uri(a.to_store)[1])
        n, tot, fps = 0, 0, []
        for p in range(meta.count):
            if p % w.size != w.rank:
                continue
            path = meta.part_path(p)
            rows = meta.parts[p].size // 24
            step_rows = 1 << 27
            for r0 in range(0, rows, step_rows):
                m = min(step_rows, rows - r0)
                buf = RD.read_to_device(path, w.device, offset=r0 * 24, length=m * 24).view(torch.int64).view(m, 3)
                tot += int((buf[:, 1] + buf[:, 2]).sum().item())
                fps.append(V.group_fingerprint([buf[:, 0], buf[:, 1], buf[:, 2]]))
                n += m
        fp = V.combine(fps)[1]
        t = torch.tensor([n, tot, fp - (1 << 64) if fp >= (1 << 63) else fp], dtype=torch.int64, device=w.device)
        if w.size > 1:
            torch.distributed.all_reduce(t)
        return [int(t[0].item()), int(t[1].item()), int(t[2].item()) & ((1 << 64) - 1)]

    step = job.step if a.direct else (store_step if a.to_store else api_step)
    if a.direct:
        job.prepare()
    for _ in range(a.warmup):
        step()
    times, res = [], None
    for _ in range(a.steps):
        dt, res = timed(w, step)
        times.append(dt)
    ok = None
    if not a.no_validate:
        if job is None:
            job = HashJoinJob(w, cfg)
        exp = job.expected()
        fp_ok = None
        if a.to_store:
            res = store_check()
            pairs_fp = job.expected_pairs("v2" if a.names else "key")
            fp_ok = res[2] == pairs_fp[1] and res[0] == pairs_fp[0]
        ok = res[0] == exp[0] and res[1] == exp[1] and fp_ok is not False
    med = sorted(times)[len(times) // 2]
    if a.names and a.name_len:
        total = 2 * rows * (a.name_len + 16)
    elif a.names:                 # Name bytes ("u" + decimal key, keys < rows) + V1 + V2 per record
        lo = lambda d: 10 ** (d - 1) if d > 1 else 0  # noqa: E731  (first key with d digits)
        ndig = sum(d * (min(rows, 10 ** d) - lo(d)) for d in range(1, 20) if lo(d) < rows)
        total = 2 * (rows * 17 + ndig)
    else:
        total = 2 * rows * 64
    if a.direct:
        js = dict(job.last)
        fallbacks = []
    else:
        last = ctx._get_executor().last_result
        js, fallbacks = dict(last["join"] or {}), last["fallbacks"]
        js["stage_seconds"] = {k: round(v, 4) for k, v in last["timings"].items()}
        if a.to_store:
            wr = last.get("write") or {}
            js["write"] = dict(GB=round(wr.get("bytes", 0) / 1e9, 2), seconds=wr.get("seconds"))
    report(w, {
        "metric": "Hash-join GB/s of input (two 100 GB tables, spill HBM -> host DRAM)",
        "value": round(total / med / 1e9, 3), "unit": "GB/s", "n_gpus": w.size, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(med * 1e3, 2), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int64",
        "data": ("synthetic gen://names tables (string key, dimension x fact; input bytes = Name + 2 x int64)"
                 if a.names else "synthetic gen://records64 row tables (dimension x fact)"),
        "validated": ok, "matches": res[0] if res else None, "all_step_ms": [round(t * 1e3, 1) for t in times],
        "pair_fingerprint_ok": fp_ok if not a.no_validate else None,
        "path": "direct (models/hashjoin.py)" if a.direct else (
            f"DryadLINQ query -> grace join stage -> {a.to_store}" if a.to_store else
            "DryadLINQ query -> fused grace join stage"),
        "fallbacks": fallbacks, "join": js,
        "config": {"model": ("R.Join(S, Name, (r, s) => (r.V2, r.V1, s.V1)).ToStore(partfile)" if a.names and a.to_store
                             else "R.Join(S, Name).Select(r.V1 + s.V1).Sum()" if a.names
                             else "R.Join(S, Key, (r, s) => (r.Key, r.V1, s.V1)).ToStore(partfile)" if a.to_store else
                             "R.Join(S, Key).Select(r.V1 + s.V1).Sum()") + " (grace hash join)", "rows_per_table": rows,
                   "row_bytes": None if a.names else 64, "input_GB": round(total / 1e9, 2),
                   "name_bytes": (a.name_len or "natural") if a.names else None,
                   "grace_join_string_bytes": a.string_bytes if a.names else None,
                   "hbm_budget_gb": a.hbm_budget_gb, "parallelism": f"dp{w.size}"}})


if __name__ == "__main__":
    main()
