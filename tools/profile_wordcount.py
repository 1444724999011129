"""Where a GPU WordCount step spends its time: wall time per step and a cProfile of the job thread.

    python tools/profile_wordcount.py [MB] [partitions]
"""
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dryad_amd as D  # noqa: E402
from dryad_amd.models.wordcount import synthetic_corpus, word_count_query  # noqa: E402


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 1000.0
    parts = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    d = tempfile.mkdtemp(prefix="dryad_wcp_")
    p = os.path.join(d, "corpus.txt")
    t = time.perf_counter()
    synthetic_corpus(p, int(mb * 1e6 / 75), vocab=50_000)
    print(f"corpus {os.path.getsize(p) / 1e6:.0f} MB in {time.perf_counter() - t:.1f}s", flush=True)
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.PartitionCount = parts
    uri = f"text://{p}?partitions={parts}"
    dict(word_count_query(ctx, uri))
    for _ in range(2):
        t = time.perf_counter()
        dict(word_count_query(ctx, uri))
        torch.cuda.synchronize()
        print(f"step {time.perf_counter() - t:.3f}s", flush=True)
    ex = ctx._get_executor()
    orig = ex.run_job
    prof = cProfile.Profile()

    def run_job(outs, handle):
        prof.enable()
        try:
            return orig(outs, handle)
        finally:
            prof.disable()
    ex.run_job = run_job
    dict(word_count_query(ctx, uri))
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(45)
    print(s.getvalue())
    os.remove(p)
    os.rmdir(d)


if __name__ == "__main__":
    main()
