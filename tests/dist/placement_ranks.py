"""Size-aware vertex placement on the SPMD GPU executor (run by tests/test_spmd.py on gloo ranks):
a partfile whose parts are heavily skewed, read with more partitions than ranks, must be placed
largest-part-first on the least-loaded rank (the reference's size-hinted scheduling,
LocalScheduler.cs:132-268) and every query over it must still equal the LocalDebug oracle."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch.distributed as dist  # noqa: E402

import dryad_amd as D  # noqa: E402
from dryad_amd import types as T  # noqa: E402
from dryad_amd.io import binary as B  # noqa: E402
from dryad_amd.io import partfile as PF  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402

SIZES = [9000, 300, 2500, 200, 200, 4000]


def main():
    w = init_world(device=os.environ.get("SPMD_DEVICE", "cpu"))
    d = os.environ["PLACEMENT_DIR"]
    meta = os.path.join(d, "skew")
    parts, v = [], 0
    for n in SIZES:
        parts.append(list(range(v, v + n)))
        v += n
    if w.rank == 0:
        base = PF.default_base(meta)
        os.makedirs(os.path.dirname(base), exist_ok=True)
        tmps = []
        for i, recs in enumerate(parts):
            p = PF.tmp_part_path(base, i, 1, 0, 0)
            B.write_records(p, T.Int32, recs)
            tmps.append(p)
        PF.commit_parts(meta, base, tmps)
    dist.barrier()
    uri = "partfile://" + meta
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    qs = {
        "groupby": lambda c: c.FromStore(uri, T.Int32).GroupBy(lambda x: x % 37, lambda k, g: (k, g.Count(), g.Sum())),
        "select_sum": lambda c: [c.FromStore(uri, T.Int32).Select(lambda x: x * 3).Sum()],
        "orderby": lambda c: c.FromStore(uri, T.Int32).Where(lambda x: x % 5 == 0).OrderBy(lambda x: -x),
    }
    W = w.size
    # LPT over SIZES (bytes = 4 per record): the largest goes to the least loaded rank first
    load, want = [0] * W, [0] * len(SIZES)
    for p in sorted(range(len(SIZES)), key=lambda q: (-SIZES[q], q)):
        r = min(range(W), key=lambda k: (load[k], k))
        want[p] = r
        load[r] += SIZES[p]
    bad = []
    for name, q in qs.items():
        g = D.DryadLinqContext(platform="gpu")
        got = q(g)
        got = got if isinstance(got, list) else list(got)
        exp = q(loc)
        exp = exp if isinstance(exp, list) else list(exp)
        res = g._get_executor().last_result
        same = got == exp if name == "orderby" else sorted(got, key=repr) == sorted(exp, key=repr)
        if not same or res.get("placement") != want:
            bad.append((name, res.get("placement"), want, same))
    allbad = [None] * W
    dist.all_gather_object(allbad, bad)
    if w.rank == 0:
        flat = [x for b in allbad for x in b]
        assert not flat, flat
        print("PLACEMENT_OK", W, want, flush=True)


if __name__ == "__main__":
    main()
    # tear the process group down before the interpreter exits: gloo's threads torn down during
    # finalisation abort the process now and then ("terminate called without an active exception")
    from dryad_amd.parallel.comm import shutdown
    shutdown()
