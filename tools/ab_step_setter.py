"""Same-box A/B of the one-GPU TeraSort step (bench.py's query path, 125 GB) across the values of
one kernel-library A/B setter (e.g. dr_terasort_gen_set_nt 0 1), interleaved, each validated.

    python tools/ab_step_setter.py <setter> <value> [<value> ...] [--steps K] [--rounds R]
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dryad_amd.models.terasort import TeraSortConfig, TeraSortQueryJob, run_steps  # noqa: E402
from dryad_amd.ops import _lib  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("setter")
    ap.add_argument("values", type=int, nargs="+")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    fn = getattr(_lib.lib(), a.setter)
    fn.argtypes = [ctypes.c_int]
    fn.restype = None
    world = init_world(device="cuda")
    job = TeraSortQueryJob(TeraSortConfig(records_per_rank=1_250_000_000), world)
    expect = job.input_checksum()
    for _ in range(2):
        job.step()
    for r in range(a.rounds):
        for v in a.values:
            fn(v)
            job.step()
            secs = run_steps(job, a.steps)
            ok = job.validate(*expect)["ok"]
            print(f"round {r} {a.setter}({v}): {1e3 * secs / a.steps:.2f} ms/step validated={ok}", flush=True)
    fn(a.values[0])


if __name__ == "__main__":
    main()
