"""Out-of-core Distinct benchmark: an all-distinct Distinct() whose RESULT exceeds the HBM budget,
streamed into the pinned host tier.

    FromStore(gen://range?count=N).Distinct().ToStore(host://distinct_out)

N int64 values (all distinct: the output is as large as the input).  Under ``--hbm-budget-gb`` the
GPU executor runs it as a streamed aggregation (runtime/stream_agg.py): chunks deduplicated on the
device into hash-bucketed running states, the largest spilled to pinned host memory, and at the
end every bucket folded once more and written straight into the host:// table
(runtime/sinks.HostSink) instead of being concatenated in HBM.  GB/s = input bytes / step time.
Validated outside the timed region: the host table's row count, value sum and an order-independent
fingerprint of every value (utils/validate.py) against the closed forms / a chunked recomputation
over 0..N-1.
"""
from __future__ import annotations

import argparse

from common import report, timed, world  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=150.0, help="input (= output) bytes, int64 values")
    ap.add_argument("--hbm-budget-gb", type=float, default=60.0)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--no-validate", action="store_true")
    a = ap.parse_args()
    w = world()
    import torch
    import dryad_amd as D
    from dryad_amd.io.providers import provider_for
    from dryad_amd.utils import validate as V
    n = int(a.gb * 1e9) // 8
    src = f"gen://range?count={n}&partitions=1&start=0"
    out = "host://distinct_out"
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = 1
    ctx.HbmBudgetBytes = int(a.hbm_budget_gb * 1e9)

    def step():
        prov = provider_for(out)
        if prov.exists(out):
            prov.delete(out)            # the previous step's pinned result goes back first
        ctx.FromStore(src).Distinct().ToStore(out, delete_if_exists=True).SubmitAndWait()

    for _ in range(a.warmup):
        step()
    times = []
    for _ in range(a.steps):
        dt, _ = timed(w, step)
        times.append(dt)
    res = ctx._get_executor().last_result
    st = [v for v in (res.get("streamed") or {}).values() if v.get("kind") == "streamed aggregation"]
    valid = None
    if not a.no_validate:
        tab = provider_for(out).get(out)["local"][0]
        got_n, got_sum, fps = 0, 0, []
        for piece in tab.device_pieces(w.device, 1 << 27):
            v = piece.cols[piece.shape.fields[0]][: piece.n].to(torch.int64)
            got_n += piece.n
            got_sum += int(v.sum())
            fps.append(V.group_fingerprint([v]))
        exp = V.combine([V.group_fingerprint([torch.arange(c, min(n, c + (1 << 27)), dtype=torch.int64,
                                                           device=w.device)]) for c in range(0, n, 1 << 27)])
        got = V.combine(fps)
        valid = dict(ok=got_n == n and got_sum == n * (n - 1) // 2 and got == exp, rows=got_n,
                     fingerprint_match=got == exp)
    med = sorted(times)[len(times) // 2]
    report(w, {
        "metric": "Out-of-core Distinct GB/s of input (all distinct: result > HBM budget, streamed to host://)",
        "value": round(n * 8 / med / 1e9, 3), "unit": "GB/s", "n_gpus": w.size, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(med * 1e3, 1), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int64", "data": "synthetic gen://range (all distinct int64)",
        "validated": None if valid is None else valid["ok"], "validation": valid,
        "fallbacks": res.get("fallbacks"), "all_step_s": [round(t, 2) for t in times],
        "config": {"model": "FromStore(gen://range).Distinct().ToStore(host://)", "rows": n,
                   "input_GB": round(n * 8 / 1e9, 1), "hbm_budget_gb": a.hbm_budget_gb,
                   "streamed": st[0] if st else None}})


if __name__ == "__main__":
    main()
