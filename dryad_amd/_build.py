"""In-tree native build for Dryad-AMD.

Two native artefacts are produced, both placed inside the package so they travel with the repo
snapshot to the GPU box:

* ``dryad_amd/_native/libdryad_kernels.so`` — every CDNA4 HIP kernel in ``csrc/kernels/*.hip``,
  compiled by ``hipcc --offload-arch=gfx950`` into one shared object with an ``extern "C"``
  launcher ABI (raw pointers + ``hipStream_t``).  Loaded with ctypes after ``import torch`` so the
  HIP runtime that torch already mapped is the one the kernels bind to (same SONAME).
* ``dryad_amd/_native/_dryad_native*.so`` — the C++ runtime (job manager state machine, message
  pump, scheduler, binary codec, partfile I/O, Rabin fingerprints) as a pybind11 module built
  with the host compiler.

Builds are incremental: a target is rebuilt only when a source or header is newer than it.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
NATIVE_DIR = Path(__file__).resolve().parent / "_native"
KERNEL_LIB = NATIVE_DIR / "libdryad_kernels.so"
ARCH = os.environ.get("DRYAD_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def _newest(paths) -> float:
    ts = [os.path.getmtime(p) for p in paths if os.path.exists(p)]
    return max(ts) if ts else 0.0


def _stale(target: Path, deps) -> bool:
    return not target.exists() or os.path.getmtime(target) < _newest(deps)


def _run(cmd, verbose):
    if verbose:
        print("[dryad-build]", " ".join(str(c) for c in cmd), file=sys.stderr)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed ({r.returncode}):\n{' '.join(map(str, cmd))}\n"
                           f"{r.stdout}\n{r.stderr}")
    return r


def build_kernels(verbose: bool = False, force: bool = False) -> Path:
    """Compile csrc/kernels/*.hip for gfx950 into one shared library (object files cached)."""
    NATIVE_DIR.mkdir(parents=True, exist_ok=True)
    objdir = ROOT / "build" / "kernels"
    objdir.mkdir(parents=True, exist_ok=True)
    srcs = sorted(glob.glob(str(CSRC / "kernels" / "*.hip")))
    hdrs = sorted(glob.glob(str(CSRC / "kernels" / "*.h")))
    objs = []
    for s in srcs:
        o = objdir / (Path(s).stem + ".o")
        if force or _stale(o, [s] + hdrs):
            _run([_hipcc(), "-c", "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC",
                  "-munsafe-fp-atomics", "-Wno-unused-result", "-I", CSRC / "kernels", s, "-o", o], verbose)
        objs.append(o)
    if force or _stale(KERNEL_LIB, objs):
        _run([_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", KERNEL_LIB], verbose)
    return KERNEL_LIB


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def runtime_lib_path() -> Path:
    return NATIVE_DIR / ("_dryad_native" + _ext_suffix())


def build_runtime(verbose: bool = False, force: bool = False) -> Path:
    """Compile the C++ runtime (csrc/runtime/*.cpp) into the pybind11 module _dryad_native."""
    import pybind11

    NATIVE_DIR.mkdir(parents=True, exist_ok=True)
    objdir = ROOT / "build" / "runtime"
    objdir.mkdir(parents=True, exist_ok=True)
    srcs = sorted(glob.glob(str(CSRC / "runtime" / "*.cpp")))
    hdrs = sorted(glob.glob(str(CSRC / "runtime" / "*.h")) + glob.glob(str(CSRC / "include" / "*.h")))
    if not srcs:
        raise RuntimeError("no runtime sources found")
    cxx = os.environ.get("CXX", "g++")
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           f"-I{CSRC / 'runtime'}", f"-I{CSRC / 'include'}"]
    flags = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
    extra = os.environ.get("DRYAD_RUNTIME_CXXFLAGS", "").split()
    objs = []
    for s in srcs:
        o = objdir / (Path(s).stem + ".o")
        if force or _stale(o, [s] + hdrs):
            _run([cxx, "-c", *flags, *extra, *inc, s, "-o", o], verbose)
        objs.append(o)
    target = runtime_lib_path()
    if force or _stale(target, objs):
        _run([cxx, "-shared", *extra, *objs, "-o", target, "-lpthread"], verbose)
    return target


LAUNCHER = NATIVE_DIR / "dryad-launch"


def build_launcher(verbose: bool = False, force: bool = False) -> Path:
    """The native per-GPU process launcher (csrc/launcher/dryad_launch.cpp)."""
    NATIVE_DIR.mkdir(parents=True, exist_ok=True)
    src = CSRC / "launcher" / "dryad_launch.cpp"
    if force or _stale(LAUNCHER, [src]):
        _run([os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", src, "-o", LAUNCHER], verbose)
    return LAUNCHER


def build_all(verbose: bool = False, force: bool = False):
    k = build_kernels(verbose, force)
    r = build_runtime(verbose, force)
    build_launcher(verbose, force)
    return k, r


if __name__ == "__main__":
    build_all(verbose=True, force="--force" in sys.argv)
