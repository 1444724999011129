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
    import torch.distributed as dist
    allbad = [bad]
    if W > 1:
        allbad = [None] * W
        dist.all_gather_object(allbad, bad)
    if w.rank == 0:
        flat = [x for b in allbad for x in b]
        assert not flat, flat
        print("FAULTS_OK", W, flush=True)


if __name__ == "__main__":
    main()
