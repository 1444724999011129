"""ctypes binding of the gfx950 kernel library (``libdryad_kernels.so``).

The library exposes an ``extern "C"`` launcher per kernel family (raw device pointers,
sizes, ``hipStream_t``; return value = ``hipError_t``).  It is loaded lazily, *after* torch so
the kernels bind to the HIP runtime torch already mapped.  On a machine with a GPU a missing
library is a hard error (no silent eager fallback); on CPU-only machines the GPU operators are
simply unavailable and the object/CPU executors are used instead.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

from .._build import KERNEL_LIB

_LOCK = threading.Lock()
_LIB = None

c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_i32 = ctypes.c_int
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
vp = ctypes.c_void_p

# name -> (restype, argtypes)
_SIGS = {
    "dr_sort_u128_workspace": (c_u64, [c_u64]),
    "dr_sort_u128": (c_i32, [vp, vp, c_u64, c_i32, c_i32, vp, vp, ctypes.POINTER(c_i32)]),
    "dr_partition_pass_u128": (c_i32, [vp, vp, c_u64, c_i32, vp, vp, vp]),
    "dr_extract_keys": (c_i32, [vp, c_u64, c_u32, c_u32, c_u32, c_u32, vp, vp]),
    "dr_gather_rows": (c_i32, [vp, vp, vp, vp, c_u64, c_u32, vp]),
    "dr_range_dest_u128": (c_i32, [vp, vp, c_u64, vp, c_u32, c_u64, c_i32, c_u32, c_u32, vp]),
    "dr_bucket_scatter_rows": (c_i32, [vp, vp, vp, c_u64, c_u32, vp, vp, vp]),
    "dr_terasort_gen": (c_i32, [vp, c_u64, c_u64, c_u64, vp]),
    "dr_terasort_check": (c_i32, [vp, c_u64, vp, vp]),
    "dr_terasort_check_desc": (c_i32, [vp, c_u64, vp, vp]),
    "dr_terasort_gen_keys": (c_i32, [vp, c_u64, c_u64, c_u64, vp, c_u32, vp, vp]),
    "dr_terasort_gen_keys64": (c_i32, [vp, c_u64, c_u64, c_u64, vp, c_u32, vp, vp]),
    "dr_terasort_gen_keys64_pitch128": (c_i32, [vp, c_u64, c_u64, c_u64, vp, c_u32, vp, vp, vp]),
    "dr_terasort_gen_hist_parts": (c_u32, [c_u64]),
    "dr_tie_fixup": (c_i32, [vp, c_u64, c_u32, vp, vp]),
    "dr_seg_sort_runs": (c_i32, [vp, c_u64, c_i32, c_u64, c_u64, vp, vp]),
    "dr_hi_range": (c_i32, [vp, c_u64, vp, vp]),
}


class NativeKernelsMissing(RuntimeError):
    pass


def _register(lib, name, sig):
    fn = getattr(lib, name)
    fn.restype, fn.argtypes = sig
    return fn


def register_signatures(sigs: dict):
    """Kernel modules add their launcher signatures here at import time."""
    _SIGS.update(sigs)
    if _LIB is not None:
        for name, sig in sigs.items():
            _register(_LIB, name, sig)


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = Path(os.environ.get("DRYAD_KERNEL_LIB", str(KERNEL_LIB)))
        if not path.exists():
            if os.environ.get("DRYAD_AUTOBUILD", "1") == "1":
                from .._build import build_kernels
                build_kernels()
            if not path.exists():
                raise NativeKernelsMissing(
                    f"{path} not built: run `python -m dryad_amd._build` (hipcc --offload-arch=gfx950)")
        l = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        for name, sig in _SIGS.items():
            _register(l, name, sig)
        _LIB = l
        return l


def available() -> bool:
    try:
        lib()
        return True
    except (NativeKernelsMissing, OSError, RuntimeError):
        return False


def stream_of(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def ptr(t: torch.Tensor | None):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"HIP kernel launcher {what} failed with hipError_t={rc}")


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    check(rc, name)
    return rc


def written(*tensors) -> None:
    """Record that a kernel wrote these existing tensors in place (through raw pointers, which
    torch does not see): bumps their version counters, so caches keyed on a tensor's version
    (column bounds in gpu/stats.py, the k-means split planes and kept sums) drop stale entries."""
    from torch.autograd.graph import increment_version
    for t in tensors:
        if t is not None:
            increment_version(t if t._base is None else t._base)
            if t._base is not None:
                increment_version(t)


def require_gpu_tensor(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise ValueError(f"{what}: expected a device (HBM) tensor, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: expected a contiguous tensor")


_HIP = None


def hip_runtime():
    """The HIP runtime torch already mapped (same SONAME as /opt/rocm's)."""
    global _HIP
    if _HIP is None:
        try:
            _HIP = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
        except OSError:
            _HIP = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"), mode=os.RTLD_GLOBAL)
        _HIP.hipHostRegister.restype = c_i32
        _HIP.hipHostRegister.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint]
        _HIP.hipHostUnregister.restype = c_i32
        _HIP.hipHostUnregister.argtypes = [vp]
        _HIP.hipMemcpyAsync.restype = c_i32
        _HIP.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, c_i32, vp]
        _HIP.hipHostGetDevicePointer.restype = c_i32
        _HIP.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
    return _HIP


def device_address(t: torch.Tensor) -> int:
    """Address of ``t``'s first element as the GPU sees it: HBM tensors as they are, page-locked
    host memory (torch-pinned or hipHostRegister'ed) through its device mapping."""
    if t.is_cuda:
        return t.data_ptr()
    out = vp()
    check(hip_runtime().hipHostGetDevicePointer(ctypes.byref(out), ctypes.c_void_p(t.data_ptr()), 0),
          "hipHostGetDevicePointer")
    return int(out.value or 0)


HIP_MEMCPY_H2D, HIP_MEMCPY_D2H = 1, 2


def memcpy_async(dst: torch.Tensor, src: torch.Tensor, stream) -> None:
    """Raw DMA copy between a device tensor and a registered (page-locked) host tensor on
    ``stream`` (a torch stream).  torch does not know hipHostRegister'ed memory is pinned and
    would stage such copies through a bounce buffer."""
    n = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() == n
    if n == 0:
        return
    kind = HIP_MEMCPY_D2H if src.is_cuda else HIP_MEMCPY_H2D
    check(hip_runtime().hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()), n, kind,
                                       ctypes.c_void_p(stream.cuda_stream)), "hipMemcpyAsync")


PREFAULT_MIN_BYTES = 64 << 20


class PinnedHostBuffer:
    """Exact-size page-locked host memory: a plain CPU tensor registered with hipHostRegister
    (torch's pinned allocator rounds requests up to a power of two, which for 100 GB spill
    buffers would double the host footprint)."""

    def __init__(self, shape, dtype=torch.uint8, prefault: bool = False):
        self.tensor = torch.empty(shape, dtype=dtype)
        nbytes = self.tensor.numel() * self.tensor.element_size()
        self.registered = False
        self.pending = None            # event after the last queued copy of the last lease
        if prefault and nbytes >= PREFAULT_MIN_BYTES:
            # first touch by torch's CPU threads before hipHostRegister; measured no faster on the
            # box (~15 GB/s of fresh pages either way, profiles/r6/r6f_pinned.log), so off by default
            self.tensor.view(-1).view(torch.uint8).zero_()
        if nbytes:
            check(hip_runtime().hipHostRegister(ctypes.c_void_p(self.tensor.data_ptr()), nbytes, 0), "hipHostRegister")
            self.registered = True

    def wait(self):
        """Block until the copies queued on the buffer by its last lease are done."""
        if self.pending is not None:
            self.pending.synchronize()
            self.pending = None

    def release(self):
        if self.registered:
            # a DMA still queued on the pages must finish before they unlock: the last lease's event,
            # or (a buffer dropped without a lease release, its copies untracked) the whole device
            if self.pending is not None:
                self.wait()
            elif torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.synchronize()
            hip_runtime().hipHostUnregister(ctypes.c_void_p(self.tensor.data_ptr()))
            self.registered = False
        self.tensor = None

    def __del__(self):
        try:
            self.release()
        except Exception:  # noqa: BLE001
            pass


# ------------------------------------------------------------------------------------------------
# Pinned host buffers reused across jobs: page-locking 25-100 GB costs seconds, so a spill tier is
# registered once per process and leased by every job that needs it (the executor's HbmPool does
# the same for HBM).
_PINNED_FREE: list = []
PINNED_KEEP = 2                    # free buffers kept for reuse (at least) ...
PINNED_KEEP_BYTES = 16 << 30       # ... and as many more as fit this many bytes (spill pieces)


class PinnedLease:
    """A ``shape`` view into a pooled page-locked buffer; ``release()`` returns it to the pool (a
    lease dropped without it is released when collected, so its queued copies stay covered)."""

    def __init__(self, buf: PinnedHostBuffer, shape, dtype):
        self._buf = buf
        n = 1
        for d in shape:
            n *= d
        esz = torch.empty(0, dtype=dtype).element_size()
        self.tensor = buf.tensor[: n * esz].view(dtype).view(*shape)

    def release(self):
        """Back to the pool, possibly with copies still queued on it (e.g. a spilled piece's copy to
        HBM): an event on the current stream marks them, and the buffer is neither unlocked nor
        handed to another lease before it has passed."""
        if self._buf is not None:
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                ev = torch.cuda.Event()
                ev.record()
                self._buf.pending = ev
            _PINNED_FREE.append(self._buf)
            while len(_PINNED_FREE) > PINNED_KEEP and \
                    sum(b.tensor.numel() for b in _PINNED_FREE) > PINNED_KEEP_BYTES:
                _PINNED_FREE.pop(0).release()
            self._buf = None
        self.tensor = None

    def __del__(self):
        try:
            self.release()
        except Exception:  # noqa: BLE001
            pass


def pinned_lease(shape, dtype=torch.uint8) -> PinnedLease:
    n = torch.empty(0, dtype=dtype).element_size()
    for d in shape:
        n *= d
    best = None
    for b in _PINNED_FREE:
        cap = b.tensor.numel()
        if n <= cap <= 2 * max(n, 1 << 20) and (best is None or cap < best.tensor.numel()):
            best = b
    if best is not None:
        _PINNED_FREE.remove(best)
        best.wait()
    else:
        best = PinnedHostBuffer((max(n, 1),))
    return PinnedLease(best, shape, dtype)
