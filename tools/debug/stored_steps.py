"""Stored TeraSort job phase by phase with a line after each (finding where a crash happens)."""
import faulthandler
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
faulthandler.enable()

from dryad_amd.models.terasort import TeraSortConfig, TeraSortStoredJob  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 3_000_000
    d = tempfile.mkdtemp(prefix="stored_dbg_")
    w = init_world(device="cuda")
    job = TeraSortStoredJob(TeraSortConfig(records_per_rank=n), w, f"partfile://{d}/in", f"partfile://{d}/out")
    print("prepare", job.prepare(), flush=True)
    print("prepare again", job.prepare(), flush=True)
    expect = job.input_checksum()
    print("checksum", expect, flush=True)
    for i in range(2):
        job.step()
        print("step", i, job.report().get("sort_path"), flush=True)
    print("validate", job.validate(*expect), flush=True)


if __name__ == "__main__":
    main()
