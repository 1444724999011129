"""WordCount (BASELINE config "WordCount via LocalJobSubmission on CPU", the reference's
canonical sample) with a device tokeniser.

    ctx.FromStore("text:///corpus.txt?partitions=P")        # LineRecord table
       .ApplyPerPartition(word_counts)                      # per-partition (word, count) partials
       .GroupBy(w => w.word, (k, g) => (k, g.Sum(c)))       # hash shuffle + final sum

``word_counts`` is a ``@device_function``: on the GPU executor the partition is a byte heap in
HBM and tokenising / grouping runs as HIP kernels (ops/text.py: byte classification + compaction,
64-bit token hashes, radix sort, segment counts, exact collision check); elsewhere it is the
plain String.Split()-style host loop, so the LocalDebug oracle and the CPU executors give the
reference answer.
"""
from __future__ import annotations

from collections import Counter

import torch

from ..attributes import device_function
from ..gpu.table import DeviceTable


def _compact_heap(t: DeviceTable) -> torch.Tensor:
    """The selected lines of a text table as one '\\n'-separated heap (e.g. the lines of a
    decoded partfile part, whose heap is the record stream with length headers between lines)."""
    if t.heap.is_cuda:
        from ..ops import channel as CH
        return CH.compact_heap(t.heap, t.cols["off"], t.cols["len"], sep=10)[0]
    ln1 = t.cols["len"] + 1
    tot = int(ln1.sum().item())
    starts = torch.cumsum(ln1, 0) - ln1
    rel = torch.arange(tot, device=t.heap.device) - torch.repeat_interleave(starts, ln1)
    src = torch.repeat_interleave(t.cols["off"], ln1) + rel
    is_sep = rel == torch.repeat_interleave(t.cols["len"], ln1)
    out = t.heap.index_select(0, torch.where(is_sep, torch.zeros_like(src), src))
    out[is_sep] = 10
    return out


@device_function
def word_counts(lines: DeviceTable) -> list:
    if lines.n == 0:
        return []
    if lines.heap is not None and lines.heap.is_cuda:
        from ..ops import text as TX
        heap = lines.heap if getattr(lines, "whole_heap", False) else _compact_heap(lines)
        t = TX.word_count_table(heap)        # (word, count) groups stay in HBM
        return t if t is not None else TX.word_count(heap)
    c = Counter()
    for ln in lines.to_objects():
        c.update((ln.Line if hasattr(ln, "Line") else ln).split())
    return list(c.items())


def word_count_query(ctx, uri: str):
    return (ctx.FromStore(uri).ApplyPerPartition(word_counts)
            .GroupBy(lambda t: t[0], lambda k, g: (k, g.Sum(lambda t: t[1]))))


def synthetic_corpus(path: str, lines: int, words_per_line: int = 12, vocab: int = 5000, seed: int = 1):
    """Zipf-ish text over a synthetic vocabulary (tests / benchmarks; no datasets offline)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    alphabet = np.array(list("abcdefghijklmnopqrstuvwxyz"))
    words = ["".join(alphabet[rng.integers(0, 26, size=int(rng.integers(2, 10)))]) for _ in range(vocab)]
    ranks = np.minimum(rng.zipf(1.3, size=lines * words_per_line) - 1, vocab - 1)
    with open(path, "w") as f:
        for i in range(lines):
            f.write(" ".join(words[r] for r in ranks[i * words_per_line:(i + 1) * words_per_line]) + "\n")
    return path
