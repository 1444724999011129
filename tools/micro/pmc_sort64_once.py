"""One compact (E64) radix sort of n generated TeraSort keys, for rocprofv3 PMC passes over the
count / scatter kernels.   python tools/micro/pmc_sort64_once.py [n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 400_000_000
    rows = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    ent = torch.empty(n, dtype=torch.int64, device="cuda")
    tmp = torch.empty(n, dtype=torch.int64, device="cuda")
    TS.generate_with_keys64(rows, 0, 7, ent)
    del rows
    S.sort_entries64(ent, tmp, 32, err=S.lookback_error())
    torch.cuda.synchronize()
    print("sorted", n, flush=True)


if __name__ == "__main__":
    main()
