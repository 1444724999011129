"""A/B of the k-means assignment kernel's prefetch depth (DR_KM_DEPTH, a build-time constant of
csrc/kernels/kmeans.hip): variant libraries built beside this file

    for d in 2 4 6; do hipcc -shared -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics \
        -Wno-unused-result -DDR_KM_DEPTH=$d -I csrc/kernels csrc/kernels/kmeans.hip \
        -o tools/micro/_km_ab/libkm_d$d.so; done

each run one full step (dr_kmeans_step_hi) on the same 125M x 128 points and K = 64 centroids,
timed with events (median of 7 after 2 warm steps: only the movers change after the first), and
the assignments compared with the in-tree library's."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.ops import kmeans as KM  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
    k = 64
    dev = torch.device("cuda")
    x = torch.empty((n, 128), dtype=torch.float32, device=dev)
    KM.generate(x)
    c = x[:: n // k][:k].clone()
    sp = KM.split_points(x)
    ws = KM.KMeansWorkspace(n, k, dev)
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_km_ab")
    libs = sorted(f for f in os.listdir(here) if f.endswith(".so")) if os.path.isdir(here) else []
    if os.environ.get("KM_AB_ONLY_IN_TREE"):
        libs = []
    ref = None
    for name in ["in-tree"] + libs:
        if name == "in-tree":
            from dryad_amd.ops import _lib
            fn = _lib.lib().dr_kmeans_step_hi
        else:
            fn = ctypes.CDLL(os.path.join(here, name)).dr_kmeans_step_hi
        fn.restype = ctypes.c_int
        vp = ctypes.c_void_p
        prev = torch.full((n,), -1, dtype=torch.int32, device=dev)
        S = torch.zeros((k, 128), dtype=torch.float64, device=dev)
        cnt = torch.zeros(k, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream().cuda_stream

        def step():
            rc = fn(vp(sp.xh.data_ptr()), vp(sp.xnorm.data_ptr()), vp(x.data_ptr()), ctypes.c_uint64(n),
                    vp(c.data_ptr()), ctypes.c_int(k), vp(ws.cnorm.data_ptr()), vp(ws.assign.data_ptr()),
                    vp(prev.data_ptr()), vp(S.data_ptr()), vp(cnt.data_ptr()), vp(ws.near.data_ptr()), vp(s))
            assert rc == 0, rc
        step()
        step()
        ts = []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            step()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        got = ws.assign[:n].clone()
        same = None if ref is None else bool(torch.equal(got, ref))
        if ref is None:
            ref = got
        print(f"{name:14s} step {sorted(ts)[3]:7.3f} ms (min {min(ts):.3f})  assignments equal to in-tree: {same}",
              flush=True)


if __name__ == "__main__":
    main()
