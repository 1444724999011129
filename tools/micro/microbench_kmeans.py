"""Time one k-means step (MFMA kernel) vs the torch (hipBLASLt GEMM + argmin + index_add) path."""
import json
import sys
import time

import os
sys_path = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, sys_path)

import torch  # noqa: E402

from dryad_amd.ops import kmeans as KM  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 50_000_000
    x = torch.empty((n, KM.DIM), dtype=torch.float32, device="cuda")
    KM.generate(x, 0, 64, 1)
    res = {"n": n}
    ks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16, 64, 128, 256, 1024]
    for k in ks:
        c = x[:k].clone()
        ws = KM.KMeansWorkspace(n, k, x.device)
        gb = n * KM.DIM * 4 / 1e9
        for tag, pl in (("planes", None), ("f32", False)) if k <= KM.PLANES_MAX_K else (("mfma", False),):
            if tag == "planes":
                t0 = time.perf_counter()
                KM.split_points(x)
                torch.cuda.synchronize()
                res["split ms (once)"] = round((time.perf_counter() - t0) * 1e3, 3)
            ms = timeit(lambda: KM.step(x, c, ws, planes=pl))
            res[f"{tag} k={k} ms"] = round(ms, 3)
            res[f"{tag} k={k} GB/s"] = round(gb / ms * 1e3, 1)
            res[f"{tag} k={k} TFLOP/s"] = round(2 * n * k * KM.DIM / ms / 1e9, 1)
        if n <= 20_000_000 and os.environ.get("KM_TORCH") == "1":
            res[f"torch k={k} ms"] = round(timeit(lambda: KM.step_reference(x, c), 2), 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
