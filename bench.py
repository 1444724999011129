#!/usr/bin/env python3
"""Headline benchmark: TeraSort GB/s sorted (whole node) on 1..8 MI355X.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

BASELINE.json metric: "GB/sec sorted (whole node), 1 TB TeraSort at 1/2/4/8 MI355X".  The
reference's TeraSort (DryadLINQ OSDI'08 §5) is weak-scaled: a fixed partition per machine
(3.87 GB), 240 machines ~ 1 TB at ~3.1 GB/s.  Here each GPU owns 125 GB (1.25e9 x 100-byte
records, 10-byte keys) so 8 GPUs sort exactly 1 TB; per-GPU work is fixed as N grows ("weak").

One step = read the input table (synthetic generator store, materialised in HBM) -> sample ->
range partition -> RCCL all-to-all-v over xGMI -> local LSD radix sort -> row gather into the
output table.  Nothing is cached between steps; the output is validated valsort-style (global
checksum, record count, in-rank order, cross-rank boundaries) after the timed region.

``--total-bytes B`` sizes the job by its total input instead (B / N per GPU, e.g. 1e12 = the
BASELINE's 1 TB).  A per-GPU share past what one GPU sorts in HBM (IN_HBM_MAX_BYTES) runs the
out-of-core path (models/terasort.TeraSortOOCJob: hybrid external sort, buckets that fit the HBM
budget stay resident, the rest spill to pinned host DRAM); the line then reports the PCIe bytes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_GBPS = 3.1   # DryadLINQ TeraSort, 240 machines, ~1 TB in ~319 s
IN_HBM_MAX_BYTES = 130e9   # per-GPU input the in-HBM sort holds (input + output + entries in 288 GB)
METRIC = "GB/sec sorted (whole node), 1 TB TeraSort at 1/2/4/8 MI355X"


# DRYAD_* variables a measured run may carry: logging / paths only.  Anything else is an A/B,
# debug or transport override of the kernels or the executor, so a headline number taken with it
# would not be the product's (``--rehearsal`` admits DRYAD_DIST_BACKEND for the shared-GPU gloo
# rehearsal of the multi-rank path and marks the line as such).
ALLOWED_ENV = {"DRYAD_LOGGING_LEVEL", "DRYAD_HOME", "DRYAD_TEMP_DIR", "DRYAD_ROCTX"}


def check_env(rehearsal: bool) -> dict:
    knobs = {k: v for k, v in os.environ.items() if k.startswith("DRYAD_") and k not in ALLOWED_ENV}
    if rehearsal:
        knobs.pop("DRYAD_DIST_BACKEND", None)
    if knobs:
        print(f"[bench] refusing to measure with engine overrides set: {knobs}", file=sys.stderr, flush=True)
        sys.exit(2)
    return {k: v for k, v in os.environ.items() if k.startswith("DRYAD_")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records-per-gpu", type=int, default=1_250_000_000)
    ap.add_argument("--total-bytes", type=float, default=None,
                    help="total input bytes over all GPUs (overrides --records-per-gpu); past the in-HBM "
                         "capacity per GPU the out-of-core path runs")
    ap.add_argument("--hbm-budget-gb", type=float, default=None, help="out-of-core path: HBM budget per GPU")
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--direct", action="store_true",
                    help="run the sort pipeline directly instead of through the DryadLINQ query API")
    ap.add_argument("--rehearsal", action="store_true",
                    help="shared-GPU gloo rehearsal of the multi-rank path (admits DRYAD_DIST_BACKEND)")
    ap.add_argument("--loopback-ranks", type=int, default=0,
                    help="run the per-rank program of a W-rank job on this one GPU, the all-to-all-v replaced by "
                         "generating the exact bytes this rank would receive (not timed); reports per-rank ms")
    ap.add_argument("--loopback-rank", type=int, default=0, help="which rank of the --loopback-ranks job to run")
    ap.add_argument("--loopback-table", choices=["terasort", "records64"], default="terasort",
                    help="with --loopback-ranks: records64 = a COLUMNAR table of 64-byte records (8 int64 columns) "
                         "ordered by --sort-key (packed into byte-keyed rows for the fine-bucket exchange)")
    ap.add_argument("--loopback-gb", type=float, default=80.0, help="with --loopback-table records64: GB per rank")
    ap.add_argument("--sort-key", default="V1", help="with --loopback-table records64: the key column")
    ap.add_argument("--descending", action="store_true",
                    help="OrderByDescending: with --loopback-table records64, or the out-of-core TeraSort (past HBM)")
    ap.add_argument("--pack-group", type=int, default=1,
                    help="with --loopback-ranks (A/B): send rounds packed per launch")
    ap.add_argument("--model-link-GBps", type=float, nargs="*", default=[300.0, 450.0],
                    help="with --loopback-ranks: MODELLED per-rank step with the all-to-all-v on a link of this many "
                         "GB/s per GPU (measured per-round pack / merge times replayed in the exchange's queue order; "
                         "labelled modelled)")
    ap.add_argument("--gen-fused", action="store_true",
                    help="N > 1 (and --loopback-ranks): no input table; the records are generated straight into "
                         "the exchange's send rows in key order (GenFusedShuffle; labelled in config.input)")
    ap.add_argument("--input", default=None,
                    help="stored-data TeraSort: read this partfile:// table of raw 100-byte rows (written from the "
                         "generator first, untimed, if absent) and write the sorted table to --output; with "
                         "--loopback-ranks: the rank's input table is read from it (one part, written if absent)")
    ap.add_argument("--output", default=None, help="with --input: the output partfile:// table")
    ap.add_argument("--rccl-one-rank", action="store_true",
                    help="rehearsal: one rank over a one-rank RCCL communicator that still runs the multi-rank "
                         "program (sampled range shuffle, fine-bucket exchange through RCCL all-to-all-v, votes) "
                         "at the full per-GPU size: the HBM working set and the RCCL path of an N-GPU run")
    args = ap.parse_args()
    env = check_env(args.rehearsal)
    if args.loopback_ranks:
        return loopback(args, env)

    import torch
    from dryad_amd.parallel.comm import init_world, shutdown
    from dryad_amd.models.terasort import (TeraSortConfig, TeraSortJob, TeraSortOOCJob, TeraSortQueryJob,
                                           TeraSortStoredJob, RECORD, run_steps)

    if args.rccl_one_rank:
        if int(os.environ.get("WORLD_SIZE", "1")) != 1:
            print("[bench] --rccl-one-rank runs without torchrun (one rank)", file=sys.stderr)
            sys.exit(2)
        from dryad_amd.parallel.comm import init_one_rank_rccl
        world = init_one_rank_rccl()
    else:
        world = init_world(device="cuda")
    if world.size != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world.size}", file=sys.stderr)
    records = args.records_per_gpu
    if args.total_bytes is not None:
        records = int(args.total_bytes / world.size) // RECORD
    ooc = records * RECORD > IN_HBM_MAX_BYTES
    cfg = TeraSortConfig(records_per_rank=records)
    t_alloc = time.perf_counter()
    stored = args.input is not None
    if stored:
        if ooc or not args.input.startswith("partfile://"):
            print("[bench] --input takes a partfile:// table that fits the in-HBM sort", file=sys.stderr)
            sys.exit(2)
        job = TeraSortStoredJob(cfg, world, args.input, args.output or args.input.rstrip("/") + "_sorted")
        prep = job.prepare()
        if world.rank == 0:
            print(f"[bench] input table: {prep}", file=sys.stderr, flush=True)
    elif ooc:
        budget = None if args.hbm_budget_gb is None else int(args.hbm_budget_gb * 1e9)
        job = TeraSortOOCJob(cfg, world, budget=budget, descending=args.descending)
    else:
        job = TeraSortJob(cfg, world) if args.direct else TeraSortQueryJob(cfg, world, gen_fused=args.gen_fused)
    if world.rank == 0:
        free, total = torch.cuda.mem_get_info(world.device)
        print(f"[bench] allocated working set in {time.perf_counter() - t_alloc:.1f}s; HBM free {free/1e9:.1f} "
              f"/ {total/1e9:.1f} GB", file=sys.stderr, flush=True)
    expect = None
    if not args.no_validate:
        expect = job.input_checksum()
        torch.cuda.empty_cache()
    for i in range(args.warmup):
        t0 = time.perf_counter()
        job.step()
        torch.cuda.synchronize()
        if world.rank == 0:
            print(f"[bench] warmup {i}: {time.perf_counter() - t0:.3f}s", file=sys.stderr, flush=True)
    secs = run_steps(job, args.steps)
    val = None
    if expect is not None:
        val = job.validate(*expect)
    total_bytes = job.bytes_per_rank * world.size
    ms = 1e3 * secs / max(args.steps, 1)
    gbps = total_bytes / 1e9 / (secs / max(args.steps, 1))
    if world.rank == 0:
        line = {
            "metric": METRIC,
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": world.size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(gbps / BASELINE_GBPS, 3),
            "dtype": "uint8",
            "data": "synthetic (gensort-style counter-generated 100-byte records, 10-byte random keys)",
            "config": {
                "model": "TeraSort 100-byte records / 10-byte key (OrderBy via range-partition + radix sort)",
                "global_batch": job.n * world.size,
                "seq_len": 100,
                "parallelism": f"dp{world.size}",
                "records_per_gpu": job.n,
                "bytes_per_gpu": job.bytes_per_rank,
                "total_bytes": total_bytes,
                "validated": None if val is None else val["ok"],
                "env": env,
                "rehearsal": bool(args.rehearsal or args.rccl_one_rank),
                "path": ("out-of-core hybrid external sort (HBM-resident buckets + pinned host DRAM)" if ooc else
                         "direct" if args.direct else
                         "DryadLINQ query -> GPU executor (fused OrderBy gang stage)" if world.size > 1 else
                         "DryadLINQ query -> GPU executor (one stage: read -> compact radix sort + gather -> output)"),
                # the input read: every record is generated once per step; with one rank into the
                # HBM input table the local sort gathers from, with several ranks straight into
                # the all-to-all send buckets (the read stage fused with the range partition)
                "input": "gen://terasort, generated in the timed step" + (
                    ": [GenFusedShuffle variant, no input table] sort entries first, then the records into the "
                    "send rows in key order (the read fused with the range partition)"
                    if world.size > 1 and args.gen_fused and not args.direct
                    else " into the HBM input table" + ("" if args.direct else
                                                         " (records at a 128-byte pitch: one aligned HBM line each)")
                    + (", then the fine-bucket exchange's send side reads it (entry sort + one row gather into "
                       "the send rows)" if world.size > 1 and not args.direct else "")),
            },
        }
        if val is not None and not val["ok"]:
            line["validation"] = val
        if args.rccl_one_rank:
            line["metric"] = METRIC + " [one-rank RCCL rehearsal of the multi-rank program]"
            line["config"]["path"] = ("DryadLINQ query -> GPU executor (fused OrderBy gang stage) over a one-rank RCCL "
                                      "communicator: sampler, fine-bucket send side, RCCL all-to-all-v rounds to "
                                      "itself, tile merge")
            line["config"]["hbm_free_after_step_GB"] = round(torch.cuda.mem_get_info(world.device)[0] / 1e9, 2)
            line["config"]["hbm_peak_allocated_GB"] = round(torch.cuda.max_memory_allocated(world.device) / 1e9, 2)
        if stored:
            line["metric"] = METRIC + " [stored-data variant: partfile in -> sort -> partfile out]"
            line["vs_baseline"] = round(gbps / BASELINE_GBPS, 3)
            line["config"]["path"] = "DryadLINQ query -> GPU executor: partfile read -> in-HBM sort -> partfile write"
            line["config"]["input"] = f"{args.input} (raw 100-byte rows, read in the timed step)"
            line["config"]["output"] = job.dst
            line["config"]["stored"] = job.report()
        elif ooc:
            line["config"]["out_of_core"] = job.report()
            if args.descending:
                line["metric"] = METRIC + " [OrderByDescending]"
                line["config"]["model"] = "TeraSort 100-byte records / 10-byte key, OrderByDescending"
            line["config"]["input"] = "gen://terasort, generated chunk by chunk in the timed step (count + partition passes)"
        elif not args.direct and not stored:
            rep = job.executor_report()
            print(f"[bench] executor: {json.dumps(rep, default=str)[:2000]}", file=sys.stderr, flush=True)
            if rep.get("exchange"):
                # per-round exchange bytes and arrival times of the last step (rank 0's view)
                line["config"]["exchange"] = rep["exchange"]
        print(json.dumps(line), flush=True)
    shutdown()
    if val is not None and not val["ok"]:
        sys.exit(3)


def loopback(args, env):
    """``--loopback-ranks W``: one rank's share of a W-GPU job, timed phase by phase on one GPU."""
    import torch
    from dryad_amd.models.terasort import TeraSortConfig, TeraSortLoopbackJob
    W, r = args.loopback_ranks, args.loopback_rank
    if W < 2 or not 0 <= r < W:
        print("[bench] --loopback-ranks needs W >= 2 and 0 <= --loopback-rank < W", file=sys.stderr)
        sys.exit(2)
    if args.loopback_table == "records64":
        return loopback_records64(args, env)
    mode = "gen-fused" if args.gen_fused else "table"
    job = TeraSortLoopbackJob(TeraSortConfig(records_per_rank=args.records_per_gpu), W, r, mode=mode,
                              input_uri=args.input, pack_group=args.pack_group)
    for i in range(args.warmup):
        job.step()
        print(f"[bench] warmup {i}: {job.ms:.2f} ms {job.phases}", file=sys.stderr, flush=True)
    ms, walls, phases = [], [], []
    for i in range(args.steps):
        t0 = time.perf_counter()
        job.step()
        walls.append(time.perf_counter() - t0)
        ms.append(job.ms)
        phases.append(job.phases)
        print(f"[bench] step {i}: {job.ms:.2f} ms {job.phases}", file=sys.stderr, flush=True)
    val = None if args.no_validate else job.validate()
    mean = sum(ms) / len(ms)
    line = {
        "metric": f"TeraSort per-rank step of a {W}-rank job (loopback on one GPU: all-to-all-v replaced)",
        "value": round(mean, 3), "unit": "ms", "higher_is_better": False, "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(mean, 3), "dtype": "uint8",
        "data": "synthetic (gensort-style counter-generated 100-byte records, 10-byte random keys)",
        "config": {"model": "TeraSort 100-byte records / 10-byte key", "records_per_rank": job.n,
                   "bytes_per_rank": job.bytes_per_rank, "ranks": W, "rank": r, "rounds": job.B,
                   "received_rows": int(job.out.shape[0]),
                   "phases_ms": {k: round(sum(p[k] for p in phases) / len(phases), 3) for k in phases[0]},
                   "per_rank_GBps": round(job.bytes_per_rank / 1e6 / mean, 1),
                   "input": (f"{args.input} (read through the chunked reader at a 128-byte pitch, timed)" if args.input
                             else "[GenFusedShuffle variant, no input table] records generated into the send rows"
                             if mode == "gen-fused" else
                             "gen://terasort generated into the rank's HBM table (128-byte pitch), timed"),
                   "wall_s_per_step_incl_simulated_exchange": round(sum(walls) / len(walls), 3),
                   # the exchange is not run here: these steps are MODELLED from the measured per-round
                   # pack / merge kernel times of the last step and an assumed per-GPU link rate
                   "modelled_exchange": ([job.model(x) for x in args.model_link_GBps]
                                         if mode == "table" and args.model_link_GBps else None),
                   "round_pack_ms": [round(x, 3) for x in job.rounds["pack_ms"]] if mode == "table" else None,
                   "round_merge_ms": [round(x, 3) for x in job.rounds["merge_ms"]],
                   "validated": None if val is None else val["ok"], "validation": val, "env": env},
    }
    print(json.dumps(line), flush=True)
    if val is not None and not val["ok"]:
        sys.exit(3)


def loopback_records64(args, env):
    """``--loopback-ranks W --loopback-table records64``: one rank's share of a W-GPU OrderBy over
    a columnar table of 64-byte records (models/records_sort.py), timed phase by phase."""
    from dryad_amd.models.records_sort import Records64LoopbackJob
    W, r = args.loopback_ranks, args.loopback_rank
    n = int(args.loopback_gb * 1e9) // 64
    job = Records64LoopbackJob(W, r, n, key=args.sort_key, descending=args.descending, pack_group=args.pack_group)
    for i in range(args.warmup):
        job.step()
        print(f"[bench] warmup {i}: {job.ms:.2f} ms {job.phases}", file=sys.stderr, flush=True)
    ms, phases = [], []
    for i in range(args.steps):
        job.step()
        ms.append(job.ms)
        phases.append(job.phases)
        print(f"[bench] step {i}: {job.ms:.2f} ms {job.phases}", file=sys.stderr, flush=True)
    val = None if args.no_validate else job.validate()
    mean = sum(ms) / len(ms)
    order = "OrderByDescending" if args.descending else "OrderBy"
    line = {
        "metric": f"{order}(r => r.{args.sort_key}) per-rank step of a {W}-rank job over a columnar table "
                  f"(loopback on one GPU: all-to-all-v replaced)",
        "value": round(mean, 3), "unit": "ms", "higher_is_better": False, "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(mean, 3), "dtype": "int64",
        "data": "synthetic gen://records64 (8 int64 columns: Key uniform in [0, 2^20), V1..V7 31-bit)",
        "config": {"model": f"records64 {order} by {args.sort_key}", "rows_per_rank": n,
                   "bytes_per_rank": job.bytes_per_rank, "row_bytes": job.rec, "key_bytes": job.lay.key_len,
                   "ranks": W, "rank": r, "rounds": job.B, "received_rows": int(job.out_cols[args.sort_key].shape[0]),
                   "phases_ms": {k: round(sum(p[k] for p in phases) / len(phases), 3) for k in phases[0]},
                   "per_rank_GBps": round(job.bytes_per_rank / 1e6 / mean, 1),
                   "input": "the rank's columnar table generated before the step (an existing hbm:// table), untimed",
                   "modelled_exchange": [job.model(x) for x in args.model_link_GBps] if args.model_link_GBps else None,
                   "round_pack_ms": [round(x, 3) for x in job.rounds["pack_ms"]],
                   "round_merge_ms": [round(x, 3) for x in job.rounds["merge_ms"]],
                   "validated": None if val is None else val["ok"], "validation": val, "env": env},
    }
    print(json.dumps(line), flush=True)
    if val is not None and not val["ok"]:
        sys.exit(3)


if __name__ == "__main__":
    main()
