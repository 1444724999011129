"""The CPU oracle suites on the GPU executor: every scenario of tests/test_api_oracle.py and
tests/test_reference_suites.py (the reference's BasicAPITests / GroupByReduceTests /
MiscBugFixTests / TypesInQueryTests / ApplyAndForkTests scenarios) runs again with the
"cluster" side being the SPMD GPU executor (3 partitions on this GPU) and the LocalDebug oracle
on the other side.  Scenarios that assert properties of the CPU process executor itself (vertex
host processes, its plan shape or its fault injection) are listed in CPU_ONLY with the reason."""
import inspect

import pytest

import helpers
import test_api_oracle as A
import test_reference_suites as R

pytestmark = pytest.mark.gpu

CPU_ONLY = {
    # the plan of the CPU executor's cluster context (the GPU executor fuses stages differently)
    "test_groupby_decomposition_is_used": "asserts the CPU plan's group_partial stage",
}


def _cases():
    out = []
    for mod in (A, R):
        for name, fn in sorted(vars(mod).items()):
            if name.startswith("test_") and inspect.isfunction(fn) and name not in CPU_ONLY:
                out.append(pytest.param(mod, name, id=f"{mod.__name__.split('_', 1)[1]}::{name}"))
    return out


@pytest.mark.parametrize("mod,name", _cases())
def test_oracle_scenario_on_gpu_executor(mod, name, tmp_path, monkeypatch):
    monkeypatch.setattr(helpers, "MODE", "gpu")
    fn = getattr(mod, name)
    params = inspect.signature(fn).parameters
    kwargs = {}
    if "tmp_path" in params:
        kwargs["tmp_path"] = tmp_path
    if any(p not in ("tmp_path",) for p in params):
        pytest.skip(f"needs fixtures {list(params)}")
    fn(**kwargs)
