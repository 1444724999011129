"""Same-box A/B of the one-GPU TeraSort step with the pitch-128 row gather copying dword-wise
(gather_fixup_kernel<25, true, 32>) or with 16-byte row loads staged through LDS
(gather_fixup_p128w_kernel), interleaved.

    python tools/ab_gather_wide.py [steps] [rounds]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dryad_amd.models.terasort import TeraSortConfig, TeraSortQueryJob, run_steps  # noqa: E402
from dryad_amd.ops import _lib  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    lib = _lib.lib()
    lib.dr_gather_fixup_set_wide.argtypes = [ctypes.c_int]
    lib.dr_gather_fixup_set_wide.restype = None
    world = init_world(device="cuda")
    job = TeraSortQueryJob(TeraSortConfig(records_per_rank=1_250_000_000), world)
    expect = job.input_checksum()
    for _ in range(2):
        job.step()
    for r in range(rounds):
        for name, wide in (("dword copy", 0), ("16-byte loads + LDS", 1), ("16-byte nontemporal loads + LDS", 2)):
            lib.dr_gather_fixup_set_wide(wide)
            job.step()
            secs = run_steps(job, steps)
            ok = job.validate(*expect)["ok"]
            print(f"round {r} {name}: {1e3 * secs / steps:.2f} ms/step validated={ok}", flush=True)
    lib.dr_gather_fixup_set_wide(1)


if __name__ == "__main__":
    main()
