import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dryad_amd.ops import channel as CH
for n, nb, kind in [(1024, 1, "i64"), (1024, 8, "i64"), (100000, 1, "i64"), (100000, 8, "i64"), (4000, 8, "i32x8")]:
    ent = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    ent[:, 1] = torch.randint(0, nb, (n,), device="cuda")
    if kind == "i64":
        cols = [torch.arange(n, device="cuda") * 10 + k for k in range(4)]
    else:
        cols = [(torch.arange(n, device="cuda") * 10 + k).to(torch.int32) for k in range(8)]
    got, cnt = CH.scatter_columns(ent, n, cols, None)
    order = torch.sort(ent[:, 1], stable=True).indices
    for k, (a, c) in enumerate(zip(got, cols)):
        b = c.index_select(0, order)
        bad = (a != b).nonzero().flatten()
        print(n, nb, kind, "col", k, "bad", bad.numel(), "first", bad[:6].tolist(), "got", a[bad[:6]].tolist(), "exp", b[bad[:6]].tolist(), "cnt", cnt[:8].tolist() if k == 0 else "", flush=True)
