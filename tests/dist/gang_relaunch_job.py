"""A three-stage SPMD job whose rank 1 is SIGKILLed in the middle of stage 1 on the gang's first
start (FaultInjection kind "kill": a real lost process, not a simulated one).  Run under
``dryad-launch --max-restarts 2 --checkpoint-dir D`` (tests/test_launch.py): the launcher stops
the gang and starts a new one; the job persisted stage 0's outputs (runtime/checkpoint.py), so
the relaunched gang resumes at stage 1 and completes oracle-equal.  Rank 0 prints the job
directory and the result check."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import dryad_amd as D  # noqa: E402
from dryad_amd.parallel.comm import init_world, shutdown  # noqa: E402


def query(c):
    pairs = c.FromEnumerable([(i % 41, i * 3 % 1009) for i in range(4000)])
    return (pairs.GroupBy(lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1])))     # stages 0 -> 1
            .Where(lambda r: r[1] > 0)
            .HashPartition(lambda r: r[2] % 7)                                                    # stage 1 -> 2
            .Select(lambda r: (r[0], r[1] * 2, r[2])))


def main():
    dev = os.environ.get("SPMD_DEVICE", "cpu")
    w = init_world(device=dev)
    g = D.DryadLinqContext(platform="gpu")
    g._props["Device"] = dev
    g.PartitionCount = w.size
    g.FaultInjection = [dict(stage=1, partition=1, version=0, kind="kill")]
    got = sorted(query(g))
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    exp = sorted(query(loc))
    ex = g._get_executor()
    res = ex.last_result
    stages = [s.name for s in ex.last_plan.stages]
    if w.rank == 0:
        print(json.dumps(dict(ok=got == exp, n=len(got), epoch=int(os.environ.get("DRYAD_GANG_EPOCH", "0")),
                              job_dir=ex.last_job_dir, recovery=[list(r) for r in res["recovery"]],
                              stages=stages)), flush=True)
    w.barrier()
    shutdown()


if __name__ == "__main__":
    main()
