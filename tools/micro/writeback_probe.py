"""Why a stored TeraSort step writes its output slower than the writer alone: isolate page-cache
write-back.  The same 8-file write (io/writer.write_device_pieces, the stored bench's output path)
is repeated back to back into fresh files, then after an ``os.sync()`` (untimed, but its own
duration says how fast the box's disk drains dirty pages), then over the previous files (the
replace-in-place pattern of the bench, old parts unlinked first), with /proc/meminfo's Dirty and
Writeback and the vm dirty limits printed around every write.

    python tools/micro/writeback_probe.py [GB] [dir]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.io import writer as WR  # noqa: E402


def meminfo() -> dict:
    out = {}
    with open("/proc/meminfo") as f:
        for ln in f:
            k, v = ln.split(":", 1)
            if k in ("MemTotal", "MemAvailable", "Dirty", "Writeback", "Cached"):
                out[k] = round(int(v.split()[0]) / 1e6, 2)          # GB (kB units)
    return out


def vm() -> dict:
    out = {}
    for k in ("dirty_ratio", "dirty_background_ratio", "dirty_bytes", "dirty_background_bytes",
              "dirty_expire_centisecs", "dirty_writeback_centisecs"):
        try:
            with open(f"/proc/sys/vm/{k}") as f:
                out[k] = int(f.read().strip())
        except OSError:
            out[k] = None
    return out


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 25
    d = sys.argv[2] if len(sys.argv) > 2 else "/tmp/wbprobe"
    os.makedirs(d, exist_ok=True)
    n = int(gb * 1e9)
    k = 8
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    bounds = [(n * j // k) for j in range(k + 1)]
    st = os.statvfs(d)
    print(f"vm {vm()}  fs free {st.f_bavail * st.f_frsize / 1e9:.1f} GB  mem {meminfo()}", flush=True)

    def write(tag, sub):
        paths = [f"{d}/{sub}_{j}" for j in range(k)]
        m0 = meminfo()
        t0 = time.perf_counter()
        WR.write_device_pieces(paths, x, bounds)
        dt = time.perf_counter() - t0
        print(f"{tag:<44} {n / 1e9 / dt:6.1f} GB/s ({dt:.2f} s)  before {m0}  after {meminfo()}", flush=True)
        return paths

    a = write("write 1 (fresh files)", "a")
    b = write("write 2 (fresh files, right after)", "b")
    t0 = time.perf_counter()
    os.sync()
    ds = time.perf_counter() - t0
    print(f"os.sync() drained the dirty pages in {ds:.2f} s  mem {meminfo()}", flush=True)
    c = write("write 3 (fresh files, after sync)", "c")
    for p in a + b:
        os.remove(p)
    write("write 4 (right after unlinking 2 x the data)", "d")
    for p in c:
        os.remove(p)
    t0 = time.perf_counter()
    os.sync()
    print(f"os.sync() {time.perf_counter() - t0:.2f} s", flush=True)
    for j in range(3):
        write(f"write {5 + j} (steady: replace the previous output)", "e")
    for f in os.listdir(d):
        os.remove(os.path.join(d, f))


if __name__ == "__main__":
    main()
