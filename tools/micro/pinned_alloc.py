"""Page-locking cost of fresh host memory: hipHostRegister of a malloc'd buffer (untouched, or
first touched in parallel by torch's CPU threads: ops/_lib.PinnedHostBuffer prefault) vs
hipHostMalloc (driver-allocated page-locked memory) vs torch's pinned allocator."""
import ctypes
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from dryad_amd.ops import _lib  # noqa: E402

torch.cuda.init()
hip = _lib.hip_runtime()
hip.hipHostMalloc.restype = ctypes.c_int
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.restype = ctypes.c_int
hip.hipHostFree.argtypes = [ctypes.c_void_p]
for gb in (2, 8, 8):
    nb = gb << 30
    for pre in (False, True):
        t0 = time.perf_counter()
        b = _lib.PinnedHostBuffer((nb,), prefault=pre)
        dt = time.perf_counter() - t0
        print(f"{gb} GB register prefault={pre}: {dt:.3f} s ({gb / dt:.1f} GB/s)", flush=True)
        b.release()
        del b
    for flags in (0, 0x4):                    # default, hipHostMallocNumaUser? (flag variants)
        p = ctypes.c_void_p()
        t0 = time.perf_counter()
        rc = hip.hipHostMalloc(ctypes.byref(p), nb, flags)
        dt = time.perf_counter() - t0
        print(f"{gb} GB hipHostMalloc flags={flags:#x}: rc={rc} {dt:.3f} s ({gb / dt:.1f} GB/s)", flush=True)
        if rc == 0:
            t1 = time.perf_counter()
            ctypes.memset(p, 0, nb)
            print(f"   first touch after hipHostMalloc: {time.perf_counter() - t1:.3f} s", flush=True)
            hip.hipHostFree(p)
    t0 = time.perf_counter()
    x = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    dt = time.perf_counter() - t0
    print(f"{gb} GB torch pin_memory: {dt:.3f} s ({gb / dt:.1f} GB/s)", flush=True)
    del x
