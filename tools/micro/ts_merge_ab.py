"""A/B of the fine-bucket receive kernel (dr_ts_tile_merge, csrc/kernels/tsmerge.hip) on one
synthetic received round: W = 8 sources, K = 131072 fine buckets (fb = 24), per-(source, bucket)
row counts Poisson(74.5) (a bucket ~596 rows, FINE_ROWS), 100-byte random rows (~7.8 GB in, 7.8 GB
out: one round of the 8-rank loopback).  Variant libraries (built beside this file, e.g. the
previous revision of tsmerge.hip) are timed against the in-tree library and their outputs
compared with it.

    python tools/micro/ts_merge_ab.py [variant ...]      # default: in-tree + every _tm_ab/*.so

A baseline variant is built from a previous revision, not kept as a source snapshot:

    mkdir -p tools/micro/_tm_ab && git show HEAD~1:csrc/kernels/tsmerge.hip > /tmp/tm_base.hip && \
    hipcc --offload-arch=gfx950 -O3 -shared -fPIC -Icsrc/kernels /tmp/tm_base.hip -o tools/micro/_tm_ab/libtm_base.so
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main():
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_tm_ab")
    have = sorted(f for f in os.listdir(here) if f.endswith(".so")) if os.path.isdir(here) else []
    want = sys.argv[1:] or ["in-tree"] + have
    W, K, fb = 8, 131072, 24
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    cnt = torch.poisson(torch.full((W, K), 74.5, device=dev), generator=g).to(torch.int32)
    n = int(cnt.sum())
    per_src = cnt.sum(1, dtype=torch.int64)
    base = torch.cumsum(per_src, 0) - per_src
    pre = (torch.cumsum(cnt.to(torch.int64), 1) - cnt.to(torch.int64) + base[:, None]).contiguous()
    col = cnt.sum(0, dtype=torch.int64)
    outoff = (torch.cumsum(col, 0) - col).contiguous()
    rows = torch.randint(0, 256, (n, 100), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty_like(rows)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    print(f"rows {n} ({n * 100 / 1e9:.2f} GB), buckets {K}, max bucket {int(col.max())}", flush=True)
    ref = None
    vp = ctypes.c_void_p
    for name in want:
        if name == "in-tree":
            from dryad_amd.ops import _lib
            fn = _lib.lib().dr_ts_tile_merge
        else:
            fn = ctypes.CDLL(os.path.join(here, name)).dr_ts_tile_merge
        fn.restype = ctypes.c_int
        s = torch.cuda.current_stream().cuda_stream

        def run():
            rc = fn(vp(rows.data_ptr()), vp(out.data_ptr()), vp(pre.data_ptr()), vp(cnt.data_ptr()),
                    vp(outoff.data_ptr()), ctypes.c_uint32(W), ctypes.c_uint32(K), ctypes.c_uint32(fb),
                    vp(flag.data_ptr()), vp(s))
            assert rc == 0, rc
        out.zero_()
        run()
        ts = []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        same = None if ref is None else bool(torch.equal(out, ref))
        if ref is None:
            ref = out.clone()
        med = sorted(ts)[3]
        print(f"{name:24s} {med:7.3f} ms (min {min(ts):.3f})  {2 * n * 100 / med / 1e9:5.2f} TB/s  "
              f"flag {int(flag.item())}  output equal to the first: {same}", flush=True)


if __name__ == "__main__":
    main()
