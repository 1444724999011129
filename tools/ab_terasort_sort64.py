"""Same-box A/B of the one-GPU TeraSort step (bench.py's query path, 125 GB) with the compact
sort's radix passes as per-pass count + scatter (dr_sort_u64) or as the single-histogram look-back
sort fed by the generator's histograms (dr_sort_u64_onesweep), interleaved.

    python tools/ab_terasort_sort64.py [steps] [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dryad_amd.models.terasort import TeraSortConfig, TeraSortQueryJob, run_steps  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    world = init_world(device="cuda")
    job = TeraSortQueryJob(TeraSortConfig(records_per_rank=1_250_000_000), world)
    expect = job.input_checksum()
    on = S.ONESWEEP_MIN
    for _ in range(2):
        job.step()
    for r in range(rounds):
        for name, thr in (("count+scatter", 1 << 62), ("onesweep+gen-hist", on)):
            S.ONESWEEP_MIN = thr
            job.step()
            secs = run_steps(job, steps)
            print(f"round {r} {name}: {1e3 * secs / steps:.2f} ms/step", flush=True)
    S.ONESWEEP_MIN = on
    print("validated:", job.validate(*expect)["ok"], flush=True)


if __name__ == "__main__":
    main()
