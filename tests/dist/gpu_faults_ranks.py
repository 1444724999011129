"""Fault injection on the SPMD GPU executor (run by tests/test_spmd.py on CPU gloo ranks and by
tests/test_gpu_multirank.py on GPU ranks): every fault kind at version 0 of partition 0 of every
stage; the results must equal the LocalDebug oracle and the recovery log must show the expected
mechanism (retry, gang restart, upstream re-execution with lineage rebuild)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import dryad_amd as D  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402

PAIRS = [(i % 53, i * 3 % 1001) for i in range(20_000)]


def queries():
    return {
        "groupby": lambda c: c.FromEnumerable(PAIRS).GroupBy(
            lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1]))),
        "orderby_take": lambda c: c.FromEnumerable(PAIRS).Select(lambda t: t[1]).OrderBy(lambda x: x).Take(300),
        "distinct_count": lambda c: [c.FromEnumerable(PAIRS).Select(lambda t: t[1] % 97).Distinct().Count()],
    }


def main():
    w = init_world(device=os.environ.get("SPMD_DEVICE", "cpu"))
    W = w.size
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    bad = []
    for kind in ("fail", "read_error", "crash", "slow:0.05"):
        for name, q in queries().items():
            g = D.DryadLinqContext(platform="gpu")
            g.PartitionCount = max(2, W)
            g.FaultInjection = [dict(stage=None, partition=0, version=0, kind=kind)]
            got = q(g)
            got = got if isinstance(got, list) else list(got)
            exp = q(loc)
            exp = exp if isinstance(exp, list) else list(exp)
            rec = g._get_executor().last_result.get("recovery") or []
            kinds = {r[0] for r in rec}
            ok = sorted(got, key=repr) == sorted(exp, key=repr)
            want = {"fail": {"retry", "gang_restart"}, "crash": {"retry", "gang_restart"},
                    "read_error": {"upstream"}, "slow:0.05": set()}[kind]
            if want and not (kinds & want):
                ok = False
            if w.rank == 0:
                print(f"[faults] {kind} {name}: {'ok' if ok else 'MISMATCH'} recovery={sorted(kinds)}", flush=True)
            if not ok:
                bad.append((kind, name, sorted(kinds)))
    if W > 1:
        bad += straggler(w, loc)
    if w.device.type == "cuda":
        bad += fused_stage_faults(w, loc)
    import torch.distributed as dist
    allbad = [bad]
    if W > 1:
        allbad = [None] * W
        dist.all_gather_object(allbad, bad)
    if w.rank == 0:
        flat = [x for b in allbad for x in b]
        assert not flat, flat
        print("FAULTS_OK", W, flush=True)


def straggler(w, loc):
    """A leaf-stage vertex stalls (slow:8 at version 0): past the outlier threshold a duplicate runs
    on an idle rank, wins, and later stages read its output from there (the reference's
    CheckForDuplicates).  The job must finish well before the straggler would have."""
    import time
    bad = []
    for name, q in queries().items():
        g = D.DryadLinqContext(platform="gpu")
        g.PartitionCount = 2 * w.size
        g.OutlierThresholdSeconds = 0.3
        g.FaultInjection = [dict(stage=0, partition=1, version=0, kind="slow:8")]   # the leaf stage
        t = time.time()
        got = q(g)
        got = got if isinstance(got, list) else list(got)
        dt = time.time() - t
        exp = q(loc)
        exp = exp if isinstance(exp, list) else list(exp)
        res = g._get_executor().last_result
        kinds = {r[0] for r in res.get("recovery") or []}
        ok = sorted(got, key=repr) == sorted(exp, key=repr)
        # on GPU ranks the OrderBy's read feeds the fused distributed sort, which takes partition
        # p on rank p: no duplicates there (the straggler is waited for)
        if not (name == "orderby_take" and w.device.type == "cuda"):
            ok = ok and "duplicate_won" in kinds and dt < 6.0 and bool(res.get("moved"))
        if w.rank == 0:
            print(f"[faults] straggler {name}: {'ok' if ok else 'MISMATCH'} {dt:.2f}s recovery={sorted(kinds)} "
                  f"moved={res.get('moved')}", flush=True)
        if not ok:
            bad.append(("straggler", name, sorted(kinds), round(dt, 2)))
    return bad


def fused_stage_faults(w, loc):
    """The same fault kinds in the fused stages (GPU ranks): the distributed OrderBy gang stage (one
    stage per rank at W = 1), the out-of-core OrderBy (host:// output) and the fused grace join;
    outputs checked exactly (order and records) and the recovery kinds as above."""
    import torch
    from dryad_amd.io.providers import provider_for
    from dryad_amd.ops import extsort as EX
    W = w.size
    bad = []
    ts = "gen://terasort?records=300000&partitions=%d&seed=5" % W
    key = lambda r: r[0:10]  # noqa: E731
    exp_sorted = list(loc.FromStore(ts).OrderBy(key))
    R = "gen://records64?count=60000&partitions=%d&keys=60000&seed=3&mode=dim" % W
    S = "gen://records64?count=60000&partitions=%d&keys=60000&seed=4" % W

    def join(c):
        return c.FromStore(R).Join(c.FromStore(S), lambda r: r[0], lambda s: s[0], lambda r, s: r[1] + s[1]).Sum()
    exp_join = join(loc)
    for kind in ("fail", "read_error", "crash"):
        want = {"fail": {"retry", "gang_restart"}, "crash": {"retry", "gang_restart"}, "read_error": {"upstream"}}[kind]
        for name in ("fused_orderby", "external_orderby", "fused_join"):
            g = D.DryadLinqContext(platform="gpu")
            g.PartitionCount = W
            g.FaultInjection = [dict(stage=None, partition=0, version=0, kind=kind)]
            if name == "fused_orderby":
                ok = list(g.FromStore(ts).OrderBy(key)) == exp_sorted
            elif name == "external_orderby":
                g.ExternalSort = True
                g.HbmBudgetBytes = 16 << 20
                uri = "host://faults_ext"
                g.FromStore(ts).OrderBy(key).ToStore(uri, delete_if_exists=True).SubmitAndWait()
                ent = provider_for(uri).get(uri)
                h, viol, first, last = EX.check_terasort_host(ent["local"][w.rank])
                rows = ent["local"][w.rank]
                mine = [bytes(x) for x in rows.rows[: rows.n].numpy()]
                allrows = [None] * W
                if W > 1:
                    import torch.distributed as dist
                    dist.all_gather_object(allrows, mine)
                else:
                    allrows = [mine]
                ok = [x for part in allrows for x in part] == exp_sorted and viol == 0
                provider_for(uri).delete(uri)
            else:
                ok = join(g) == exp_join
            rec = g._get_executor().last_result.get("recovery") or []
            kinds = {r[0] for r in rec}
            # one rank: the OrderBy is one stage reading its own source, no channel to fail
            one_stage = W == 1 and name == "fused_orderby" and kind == "read_error"
            if not one_stage and not (kinds & want):
                ok = False
            if w.rank == 0:
                print(f"[faults] {kind} {name}: {'ok' if ok else 'MISMATCH'} recovery={sorted(kinds)}", flush=True)
            if not ok:
                bad.append((kind, name, sorted(kinds)))
    torch.cuda.synchronize()
    return bad


if __name__ == "__main__":
    main()
    # tear the process group down before the interpreter exits: gloo's threads torn down during
    # finalisation abort the process now and then ("terminate called without an active exception")
    from dryad_amd.parallel.comm import shutdown
    shutdown()
