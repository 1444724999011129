"""Compare the device chains of the variable-length boundary scan (csrc/kernels/varscan.hip)
with a CPU re-implementation on the first chunks of the codec_bw data set."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dryad_amd import types as T  # noqa: E402
from dryad_amd.io import binary as B  # noqa: E402
from dryad_amd.ops import codec as CD  # noqa: E402

BAD = -1
K = 6


def step(b, p, n, sizes):
    for sz in sizes:
        if sz:
            p += sz
            continue
        if p >= n:
            return BAD
        u = int(b[p])
        if u < 0x80:
            p += 1
        else:
            if p + 4 > n:
                return BAD
            u = ((u & 0x7f) << 24) | (int(b[p + 1]) << 16) | (int(b[p + 2]) << 8) | int(b[p + 3])
            if u < 0x80:
                return BAD
            p += 4
        if p >= n:
            return BAD
        nb = int(b[p])
        wide = (u + 1) * 3 >= 0x80
        if nb < 0x80:
            if wide:
                return BAD
            p += 1
        else:
            if not wide or p + 4 > n:
                return BAD
            nb = ((nb & 0x7f) << 24) | (int(b[p + 1]) << 16) | (int(b[p + 2]) << 8) | int(b[p + 3])
            p += 4
        if nb < u or nb > 3 * u:
            return BAD
        p += nb
    return p if p <= n else BAD


def chain(b, n, c, C, sizes):
    s0, s1 = c * C, min(c * C + C, n)
    p, start, run, locked = s0, s0, [], c == 0
    pos = []
    while p < s1:
        q = step(b, p, n, sizes)
        if q == BAD or (not locked and q - p > C):
            if locked:
                break
            run, start = [], start + 1
            p = start
            continue
        if locked:
            pos.append(p)
        else:
            run.append(p)
            if len(run) == K:
                locked = True
                pos += run
        p = q
    if not locked and run and p >= s1:
        pos += run
        locked = True
    return (p if locked and p >= s1 else BAD), pos


def main():
    rng = np.random.default_rng(1)
    alpha = "abcdefghijklmnopqrstuvwxyz"
    vdt = T.RecordT([("k", T.Int64), ("s", T.String), ("x", T.Float64)], tuple)
    recs = [(i, "".join(alpha[j] for j in rng.integers(0, 26, size=int(rng.integers(12, 41)))), i * 0.5)
            for i in range(200_000)]
    blob = np.frombuffer(B.encode_records(vdt, recs), dtype=np.uint8)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    part = np.tile(blob, reps)
    buf = torch.from_numpy(part).cuda()
    dbg = {}
    got = CD.block_index_device(buf, vdt, debug=dbg)
    print("scan:", CD.LAST_SCAN, "result None" if got is None else f"{got[0]} records")
    ex = dbg["exitp"].cpu().numpy()
    sy = dbg["sync"].cpu().numpy()
    bits = dbg["bits"].cpu().numpy().view(np.uint32)
    good = dbg["good"].cpu().numpy()
    n = len(part)
    b = part                                             # numpy indexing: no list of 10e9 ints
    C = CD.VARSCAN_CHUNK
    bad_idx = np.nonzero(~good)[0]
    print("irregular chunks:", len(bad_idx), "first:", bad_idx[:20].tolist())
    if len(bad_idx):
        exb, syb = ex[bad_idx], sy[bad_idx]
        far = (syb >= 0) & (syb // C != bad_idx + 1)
        print("  exit < 0:", int((exb < 0).sum()), " sync < 0:", int(((exb >= 0) & (syb < 0)).sum()),
              " sync past the next chunk:", int(far.sum()))
        print("  irregular chunk positions (bytes):", (bad_idx[:10] * C).tolist())
    mism = 0
    for c in list(range(0, 40)) + bad_idx[:10].tolist():
        c = int(c)
        e, pos = chain(b, n, c, C, [8, 0, 8])
        w0, w1 = (c * C) >> 5, (min(c * C + C, n) + 31) >> 5
        dev = [((w << 5) + k) for w in range(w0, w1) for k in range(32) if (bits[w] >> k) & 1]
        ok = e == ex[c] and dev == pos
        if not ok:
            mism += 1
            print(f"chunk {c}: cpu exit {e} dev exit {ex[c]} sync {sy[c]}; cpu {len(pos)} positions {pos[:6]}, "
                  f"dev {len(dev)} positions {dev[:6]}")
    print("mismatching chunks:", mism)
    # the exit walks of the first irregular chunks, redone on the host over the device's bits
    for c in bad_idx[:8].tolist():
        p, k, y = int(ex[c]), 0, BAD
        while p != BAD:
            if p >= n:
                y = n if p == n else BAD
                break
            if (int(bits[p >> 5]) >> (p & 31)) & 1:
                y = p
                break
            k += 1
            if k > 70000:
                y = -2
                break
            p = step(b, p, n, [8, 0, 8])
        print(f"walk of chunk {c}: host sync {y} (chunk {y // C if y >= 0 else None}, {k} steps), device sync {sy[c]}, "
              f"exit {ex[c]}")


if __name__ == "__main__":
    main()
