"""Page-locking cost of a fresh host buffer: hipHostRegister of untouched pages vs pages first
touched in parallel by torch's CPU threads (ops/_lib.PinnedHostBuffer prefault)."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from dryad_amd.ops import _lib  # noqa: E402

torch.cuda.init()
for gb in (2, 8):
    for pre in (False, True, False, True):
        t0 = time.perf_counter()
        b = _lib.PinnedHostBuffer((gb << 30,), prefault=pre)
        dt = time.perf_counter() - t0
        print(f"{gb} GB prefault={pre}: {dt:.3f} s ({gb / dt:.1f} GB/s)", flush=True)
        b.release()
        del b
