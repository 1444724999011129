"""Per-variant kmeans_assign_kernel times from a rocprofv3 --kernel-trace of km_depth_ab.py: the
dispatches in order, 9 per variant (2 warm + 7 timed steps), variants in the tool's order."""
import csv
import os
import sys


def main():
    trace = sys.argv[1]
    names = ["in-tree"] + sorted(f for f in os.listdir(os.path.join(os.path.dirname(__file__), "_km_ab"))
                                 if f.endswith(".so"))
    rows = [r for r in csv.DictReader(open(trace)) if "kmeans_assign_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for i, nm in enumerate(names):
        ts = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[9 * i: 9 * i + 9])
        if ts:
            print(f"{nm:22s} kmeans_assign_kernel median {ts[len(ts) // 2]:.3f} ms  min {ts[0]:.3f} ms "
                  f"({32e9 / 1e12 / (ts[len(ts) // 2] / 1e3):.2f} TB/s of the 32 GB bf16 plane)")


if __name__ == "__main__":
    main()
