"""Standalone re-run of one failed GPU vertex from its restart record (reference
``DumpRestartCommand`` + the ``--cmd`` vertex controller, dvertexpncontrol.cpp:348-736,
dvertexcmdlinecontrol.cpp:926-1030; JobBrowser ``LocalDebuggingAndProfiling.cs:97-160``).

    python -m dryad_amd.tools.replay JOB_DIR/log/rerun/vertex-V.v [--device cuda|cpu] [--show N]

The GPU executor writes, for every failed vertex attempt, the inputs that were delivered to it:
device tables as tensor files (loaded with ``torch.load(weights_only=True)``) plus a JSON layout,
host record lists as pickles written by this framework, and the job's plan.  The replay rebuilds
the tables on the chosen device and runs the stage's operator program for that partition alone, so
a failure can be reproduced (and debugged / profiled) without re-running the job.
"""
from __future__ import annotations

import argparse
import json
import os
import pickle
import sys

import torch


def _shape_json(sh):
    from ..gpu.table import PartialMeta
    py = sh.pytype
    if isinstance(py, PartialMeta):
        pyj = {"partial": [py.nkeys, list(py.kinds), py.key_form, bool(getattr(py, "raw", False))]}
    elif py is None:
        pyj = None
    elif isinstance(py, type):
        pyj = {"class": f"{py.__module__}:{py.__qualname__}"}
    else:
        from .. import types as T
        pyj = {"dtype": T.dtype_to_json(py)}
    return dict(kind=sh.kind, fields=list(sh.fields), pytype=pyj, key_off=sh.key_off, key_len=sh.key_len)


def _shape_from(d):
    from ..gpu.table import PartialMeta, Shape
    from .. import types as T
    pj = d.get("pytype")
    py = None
    if pj and "partial" in pj:
        py = PartialMeta(pj["partial"][0], tuple(pj["partial"][1]), pj["partial"][2],
                         bool(pj["partial"][3]) if len(pj["partial"]) > 3 else False)
    elif pj and "class" in pj:
        py = T._lookup_class(pj["class"])
        if py is None and pj["class"] in ("builtins:str",):
            py = str
        if py is None and pj["class"].endswith(":LineRecord"):
            py = T.LineRecord
    elif pj and "dtype" in pj:
        py = T.dtype_from_json(pj["dtype"])
    return Shape(d["kind"], list(d["fields"]), py, d.get("key_off", 0), d.get("key_len", 0))


def dump(job_dir, plan, stage, partition, vertex, version, streams, error):
    """Write the restart record (called by the GPU executor on a failed attempt)."""
    from ..gpu.table import DeviceTable
    d = os.path.join(job_dir, "log", "rerun", f"vertex-{vertex}.{version}")
    os.makedirs(d, exist_ok=True)
    pk = os.path.join(job_dir, "plan.pkl")
    if not os.path.exists(pk):
        import cloudpickle
        with open(pk, "wb") as f:
            cloudpickle.dump(plan, f)
    inputs = None
    if streams is not None:
        inputs = []
        for ii, inp in enumerate(streams):
            files = []
            for k, x in enumerate(inp):
                base = os.path.join(d, f"in{ii}_{k}")
                if isinstance(x, DeviceTable):
                    tensors = {"col:" + c: v.detach().cpu() for c, v in x.cols.items()}
                    if x.rows is not None:
                        tensors["rows"] = x.rows.detach().cpu()
                    if x.heap is not None:
                        tensors["heap"] = x.heap.detach().cpu()
                    for f_, h in x.strs.items():
                        tensors["str:" + f_] = h.detach().cpu()
                    torch.save(tensors, base + ".pt")
                    with open(base + ".json", "w") as f:
                        json.dump(dict(n=x.n, shape=_shape_json(x.shape), cols=list(x.cols)), f)
                    files.append(os.path.basename(base) + ".pt")
                else:
                    with open(base + ".pkl", "wb") as f:
                        pickle.dump(x, f)
                    files.append(os.path.basename(base) + ".pkl")
            inputs.append(files)
    with open(os.path.join(d, "cmd.json"), "w") as f:
        json.dump(dict(job=job_dir, stage=stage.id, stage_name=stage.name, partition=partition, vertex=vertex,
                       version=version, inputs=inputs, error=error), f, indent=1)
    return d


def load_inputs(d, cmd, device):
    from ..gpu.table import DeviceTable
    streams = []
    for files in cmd["inputs"]:
        inp = []
        for name in files:
            path = os.path.join(d, name)
            if name.endswith(".pt"):
                t = torch.load(path, weights_only=True)
                with open(path[:-3] + ".json") as f:
                    meta = json.load(f)
                cols = {c: t["col:" + c].to(device) for c in meta["cols"]}
                strs = {k[4:]: v.to(device) for k, v in t.items() if k.startswith("str:")}
                inp.append(DeviceTable(meta["n"], _shape_from(meta["shape"]), cols,
                                       rows=t["rows"].to(device) if "rows" in t else None,
                                       heap=t["heap"].to(device) if "heap" in t else None, strs=strs))
            else:
                with open(path, "rb") as f:          # written by this framework's own GPU executor
                    inp.append(pickle.load(f))
        streams.append(inp)
    return streams


def replay(d, device="cuda"):
    """-> (ok, output or exception)."""
    import cloudpickle  # noqa: F401  (reducers of the pickled plan's lambdas)
    import dryad_amd as D
    from ..parallel.comm import World
    from ..runtime.gpu_executor import GpuJobRunner
    with open(os.path.join(d, "cmd.json")) as f:
        cmd = json.load(f)
    if cmd.get("inputs") is None:
        raise RuntimeError("the restart record has no persisted inputs (larger than RerunInputsMaxBytes)")
    with open(os.path.join(cmd["job"], "plan.pkl"), "rb") as f:
        plan = pickle.load(f)                        # this framework's own plan file
    dev = torch.device(device if device != "cuda" or torch.cuda.is_available() else "cpu")
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.AllowHostFallback = True
    runner = GpuJobRunner(ctx, plan, World(0, 1, 0, dev, None))
    st = plan.stages[cmd["stage"]]
    streams = load_inputs(d, cmd, dev)
    try:
        return True, runner.run_vertex(st, cmd["partition"], cmd["version"], streams, inject=False)
    except Exception as e:  # noqa: BLE001
        return False, e


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m dryad_amd.tools.replay")
    ap.add_argument("rerun_dir")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--show", type=int, default=5)
    a = ap.parse_args(argv)
    with open(os.path.join(a.rerun_dir, "cmd.json")) as f:
        cmd = json.load(f)
    print(f"replaying {cmd['stage_name']}[{cmd['partition']}] v{cmd['version']} (original error: {cmd['error']})")
    ok, out = replay(a.rerun_dir, a.device)
    if not ok:
        print(f"vertex failed again: {type(out).__name__}: {out}")
        return 1
    from ..runtime.gpu_executor import _to_objects
    recs = _to_objects(out) if not isinstance(out, list) else out
    print(f"vertex completed: {len(recs)} records; first {min(a.show, len(recs))}: {recs[:a.show]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
