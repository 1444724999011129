#!/usr/bin/env python3
"""Per-iteration time of local k-means iterations, eager launches vs one hipGraph replay
(dryad_amd/runtime/hipgraph.py), over point counts where launches do / do not matter."""
import sys
import time

import torch

sys.path.insert(0, ".")
from dryad_amd.ops import kmeans as KM                      # noqa: E402
from dryad_amd.runtime.hipgraph import KMeansGraph          # noqa: E402

ITERS = 64


def eager(x, c0, iters):
    ws = KM.KMeansWorkspace(x.shape[0], c0.shape[0], x.device)
    c = c0.clone()
    for _ in range(iters):
        s, n, _ = KM.step(x, c, ws)
        c = KM.update(c, s, n)
    return c


def best(fn, reps=3):
    out = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out = min(out, time.perf_counter() - t)
    return out


def main():
    for n in (100_000, 1_000_000, 4_000_000, 32_000_000):
        for k in (16, 64):
            x = KM.generate(torch.empty((n, KM.DIM), dtype=torch.float32, device="cuda"))
            c0 = x[:k].clone()
            eager(x, c0, 2)
            te = best(lambda: eager(x, c0, ITERS))
            g = KMeansGraph(x, c0, unroll=16)
            tg = best(lambda: (g.restart(), g.run(ITERS)))
            ce, cg = eager(x, c0, ITERS), (g.restart(), g.run(ITERS))[1]
            torch.cuda.synchronize()
            d = (ce - cg).abs().max().item()
            print(f"n={n:>10,} K={k:>3}: eager {1e6 * te / ITERS:8.1f} us/iter, hipGraph {1e6 * tg / ITERS:8.1f} "
                  f"us/iter ({te / tg:4.2f}x), max |dc| {d:.2e}", flush=True)
            del x, g


if __name__ == "__main__":
    main()
