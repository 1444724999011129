"""Cost of persisting one rank's stage output for a gang relaunch (runtime/checkpoint.py): a
``--gb`` GB device row table saved through the native part writer and loaded back, into
/dev/shm (the relaunching launcher's default tier) and into a disk directory; reports GB/s and
checks the loaded rows byte for byte (TeraSort checksum).

    python tools/ckpt_bench.py --gb 25 [--dirs /dev/shm /tmp]
"""
import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dryad_amd.gpu.table import DeviceTable  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402
from dryad_amd.runtime import checkpoint as CK  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=25.0)
    ap.add_argument("--dirs", nargs="*", default=["/dev/shm", "/tmp"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = int(a.gb * 1e9) // 100
    rows = torch.empty((n, 100), dtype=torch.uint8, device=dev)
    TS.generate(rows, 0, 77)
    ref = TS.check(rows).clone()
    t = DeviceTable.from_rows(rows, 0, 10)
    out = []
    for d in a.dirs:
        st = os.statvfs(d)
        free = st.f_bavail * st.f_frsize
        if free < 1.2 * n * 100:
            out.append(dict(dir=d, skipped=f"{free / 1e9:.1f} GB free"))
            continue
        root = os.path.join(d, f"ckpt_bench_{os.getpid()}")
        ck = CK.StageCheckpoint(root, "job0000-bench")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nb = ck.save(1, 0, t)
        t1 = time.perf_counter()
        back = ck.load(1, 0, dev)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ok = torch.equal(TS.check(back.rows), ref) and back.n == n
        del back
        shutil.rmtree(root, ignore_errors=True)
        out.append(dict(dir=d, GB=round(nb / 1e9, 2), persist_ms=round((t1 - t0) * 1e3, 1),
                        persist_GBps=round(nb / 1e9 / (t1 - t0), 2), load_ms=round((t2 - t1) * 1e3, 1),
                        load_GBps=round(nb / 1e9 / (t2 - t1), 2), verified=bool(ok),
                        files=CK.PIECE and len([0 for _ in range(min(8, -(-nb // CK.PIECE)))])))
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps(dict(metric="stage checkpoint persist / load", results=out)), flush=True)


if __name__ == "__main__":
    main()
