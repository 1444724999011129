"""Per-kernel HBM bytes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (rocpd databases):
summed kilobytes per kernel name, with the kernels' summed duration and the implied GB/s.

    python tools/pmc_bytes.py fetch.db write.db [--top N]
"""
import argparse
import sqlite3
from collections import defaultdict


def load(db):
    c = sqlite3.connect(db)
    out = defaultdict(lambda: [0.0, 0, 0])        # name -> [KB, ns, dispatches]
    for name, kb, dur in c.execute("select kernel_name, value, duration from counters_collection"):
        n = name.replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0][:60]
        o = out[n]
        o[0] += kb
        o[1] += dur
        o[2] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    f, w = load(a.fetch), load(a.write)
    names = sorted(f, key=lambda k: -f[k][1])[: a.top]
    print(f"{'kernel':60s} {'calls':>5s} {'ms':>9s} {'read GB':>9s} {'write GB':>9s} {'TB/s':>6s}")
    for n in names:
        kb_r, ns, calls = f[n]
        kb_w = w.get(n, [0.0, 0, 0])[0]
        gb_r, gb_w = kb_r * 1024 / 1e9, kb_w * 1024 / 1e9
        ms = ns / 1e6
        print(f"{n:60s} {calls:5d} {ms:9.2f} {gb_r:9.2f} {gb_w:9.2f} {(gb_r + gb_w) / max(ms, 1e-9):6.2f}")


if __name__ == "__main__":
    main()
