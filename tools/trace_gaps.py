"""Kernel timeline of a rocprofv3 rocpd database: every kernel in start order with the idle gap
before it, and the total busy / idle time between the first and last kernel of the window.

    python tools/trace_gaps.py gpurun_out/prof_ts/.../run_results.db [--last N] [--min-gap-us G]

Used to find host overhead between the kernels of one bench step (GPU idle while Python plans or
synchronises)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=60, help="kernels at the end of the run to show")
    ap.add_argument("--min-gap-us", type=float, default=0.0, help="only list kernels after a gap this long")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
    rows = sorted(c.execute(f"select {name_col}, start, end from kernels").fetchall(), key=lambda r: r[1])
    rows = rows[-a.last:]
    busy = idle = 0
    prev_end = None
    for name, s, e in rows:
        n = name.replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0][:70]
        gap = 0 if prev_end is None else max(0, s - prev_end)
        busy += e - s
        idle += gap
        if gap / 1e3 >= a.min_gap_us:
            print(f"gap {gap / 1e3:10.1f} us  run {(e - s) / 1e3:10.1f} us  {n}")
        prev_end = max(prev_end or 0, e)
    span = rows[-1][2] - rows[0][1] if rows else 0
    print(f"window: {len(rows)} kernels, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle {idle / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
