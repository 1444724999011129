"""Send side of the fine-bucket multi-rank TeraSort (one rank of W), phase by phase.

    python tools/micro/ts_send_ab.py [W] [rows]

Times, at full size: E64 entries from the generator (with histograms), the look-back sort on the
top 24 key bits, the fine-bucket starts, and the record generation into the send rows three ways
(one launch over all entries, one launch per key range as pack_gen_fine does, and the int32-offset
generator of the old bucket pack for comparison).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


def timed(fn, reps=2):
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1)
        best = t if best is None else min(best, t)
    return best


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    W = int(args[0]) if args else 8
    n = int(float(args[1])) if len(args) > 1 else 1_250_000_000
    dev = torch.device("cuda", 0)
    seed = 7
    e = torch.empty(n, dtype=torch.int64, device=dev)
    tmp = torch.empty(n, dtype=torch.int64, device=dev)
    out = torch.empty((n, 100), dtype=torch.uint8, device=dev)
    fb = RS.fine_bits(n * W)
    win = 8 * ((fb + 7) // 8)
    print(f"rows {n:.3g}, W={W}, fb={fb}, sort bits {win}", flush=True)
    holder = {}
    t = timed(lambda: holder.update(h=TS.gen_entries64(e, 0, seed)))
    print(f"entries + histograms        {t:8.2f} ms", flush=True)
    err = S.lookback_error()

    def srt():
        h = TS.gen_entries64(e, 0, seed)
        holder["s"] = S.sort_entries64(e, tmp, win, gen_hist=h, err=err)
    t2 = timed(srt)
    print(f"look-back sort ({win} bits)   {t2 - t:8.2f} ms  err={int(err.item())}", flush=True)
    s = holder["s"]
    t = timed(lambda: holder.update(st=TS.fine_starts(s, fb)))
    print(f"fine starts                 {t:8.2f} ms", flush=True)
    t = timed(lambda: TS.gen_gather64(out, s, 0, seed))
    print(f"gen_gather64, one launch    {t:8.2f} ms", flush=True)
    B = RS.pipeline_subs(n * 100, W)
    cuts = [(n * j) // (W * B) for j in range(W * B + 1)]

    def per_range():
        for j in range(W * B):
            TS.gen_gather64(out[cuts[j]: cuts[j + 1]], s[cuts[j]: cuts[j + 1]], 0, seed)
    t = timed(per_range)
    print(f"gen_gather64, {W * B} launches  {t:8.2f} ms", flush=True)
    R = 16
    cut16 = [(n * j) // R for j in range(R + 1)]

    def per_round_plain():
        for j in range(R):
            TS.gen_gather64(out[cut16[j]: cut16[j + 1]], s[cut16[j]: cut16[j + 1]], 0, seed)
    t = timed(per_round_plain)
    print(f"gen_gather64, {R} launches, no segments  {t:8.2f} ms", flush=True)
    # the pack's layout: round b = W segments (ranges r * B + b) of the key-ordered entries
    W8 = W
    segs = []
    for b in range(R):
        rows_b, seg = 0, []
        for r in range(W8):
            g = r * R + b
            a0, a1 = (n * g) // (W8 * R), (n * (g + 1)) // (W8 * R)
            seg.append([rows_b, a0])
            rows_b += a1 - a0
        segs.append((rows_b, torch.tensor(seg, dtype=torch.int64, device=dev)))
    starts = [0]
    for rows_b, _ in segs:
        starts.append(starts[-1] + rows_b)

    def per_round_segs():
        for b in range(R):
            TS.gen_gather64(out[starts[b]: starts[b + 1]], s, 0, seed, seg=segs[b][1], n=segs[b][0])
    t = timed(per_round_segs)
    print(f"gen_gather64, {R} launches x {W8} segments  {t:8.2f} ms", flush=True)
    idx = tmp.view(torch.int32)[:n]
    idx.copy_((s & 0xFFFFFFFF).to(torch.int32))
    t = timed(lambda: TS.gen_gather(out, idx, 0, seed))
    print(f"gen_gather (int32 offsets)  {t:8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
