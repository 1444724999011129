"""WordCount benchmark (BASELINE.json config "WordCount via LocalJobSubmission on CPU (plumbing,
runs without a GPU)"): MB/s of text counted, validated against collections.Counter.

    python benchmarks/wordcount.py [--mb 256] [--procs 4] [--partitions 8] [--gpu]

Default: the CPU process executor (LocalJobSubmission analog, ``--procs`` worker processes), the
reference's own sample.  ``--gpu``: the same query through the GPU executor with the device
tokeniser (ops/text.py).  The corpus is synthetic (Zipf-ish words over a generated vocabulary);
it is written once, outside the timed region; every timed step reads it from the file system.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=256.0)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    import dryad_amd as D
    from dryad_amd.models.wordcount import synthetic_corpus, word_count_query
    d = tempfile.mkdtemp(prefix="dryad_wc_")
    p = os.path.join(d, "corpus.txt")
    lines = int(a.mb * 1e6 / 75)            # ~75 bytes per 12-word line
    synthetic_corpus(p, lines, vocab=50_000)
    size = os.path.getsize(p)
    uri = f"text://{p}?partitions={a.partitions}"
    ctx = D.DryadLinqContext(platform="gpu") if a.gpu else D.DryadLinqContext(a.procs)
    if a.gpu:
        ctx.PartitionCount = a.partitions
    res = dict(word_count_query(ctx, uri))          # warmup (worker start, kernel load)
    times = []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        res = dict(word_count_query(ctx, uri))
        times.append(time.perf_counter() - t0)
    with open(p) as f:
        ok = res == dict(Counter(f.read().split()))
    med = sorted(times)[len(times) // 2]
    print(json.dumps({
        "metric": "WordCount MB/s of text (LocalJobSubmission on CPU)" if not a.gpu else "WordCount MB/s of text (GPU executor)",
        "value": round(size / med / 1e6, 2), "unit": "MB/s", "steps": a.steps, "seconds_per_step": round(med, 3),
        "all_step_s": [round(t, 4) for t in times],
        "higher_is_better": True, "validated": ok, "words": len(res), "bytes": size,
        "data": "synthetic Zipf-ish corpus (models/wordcount.synthetic_corpus)",
        "config": {"executor": "gpu" if a.gpu else f"process x{a.procs}", "partitions": a.partitions}}))
    os.remove(p)
    os.rmdir(d)
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
