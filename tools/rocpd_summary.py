"""Summarise a rocprofv3 rocpd SQLite database: per-kernel total / count / mean time.

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--last-fraction F] [--csv out.csv]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for name, s, e in rows:
        n = name.replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0]
        if len(n) > 90:
            n = n[:90]
        t, k = agg.get(n, (0, 0))
        agg[n] = (t + (e - s), k + 1)
    total = sum(t for t, _ in agg.values())
    out = sorted(agg.items(), key=lambda kv: -kv[1][0])
    lines = ["kernel,calls,total_ms,mean_us,pct"]
    for n, (t, k) in out[: a.top]:
        lines.append(f"\"{n}\",{k},{t / 1e6:.3f},{t / k / 1e3:.1f},{100 * t / total:.1f}")
    txt = "\n".join(lines)
    print(txt)
    print(f"# total kernel time {total / 1e6:.1f} ms over {len(rows)} dispatches")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
