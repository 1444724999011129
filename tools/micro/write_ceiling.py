"""HBM write-stream ceiling vs the gen://records64 column generator (csrc/kernels/generators.hip):
4 int64 columns of 1.25e9 rows (40 GB) written by torch fill_, by a 16-byte-store copy_, and by
gen_records64 (the GroupBy bench's input).  Min of 5 timed repeats each."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from dryad_amd.ops import relational as R  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000_000
cols = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(4)]
src = torch.empty(n, dtype=torch.int64, device="cuda")
src.fill_(7)


def timed(fn, label, nbytes):
    ts = []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    t = min(ts[1:])
    print(f"{label:34s} {t:7.2f} ms  {nbytes / t / 1e9:6.2f} TB/s", flush=True)


B = 4 * n * 8
timed(lambda: [c.fill_(3) for c in cols], "fill_ 4 columns (write only)", B)
timed(lambda: [c.zero_() for c in cols], "zero_ 4 columns (write only)", B)
timed(lambda: [c.copy_(src) for c in cols], "copy_ 4 columns (read + write)", 2 * B)
timed(lambda: R.gen_records64(cols, 0, 1 << 30, 11), "gen_records64 4 columns", B)
