"""The CPU oracle suites on the GPU executor: every scenario of tests/test_api_oracle.py and
tests/test_reference_suites.py (the reference's BasicAPITests / GroupByReduceTests /
MiscBugFixTests / TypesInQueryTests / ApplyAndForkTests scenarios) runs again with the
"cluster" side being the SPMD GPU executor (3 partitions on this GPU) and the LocalDebug oracle
on the other side.  Scenarios that assert properties of the CPU process executor itself (vertex
host processes, its plan shape or its fault injection) are listed in CPU_ONLY with the reason."""
import collections
import inspect
import os

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


# Host fallbacks a scenario may take on the GPU executor, each with the reason its operator cannot
# run on the device.  Any other fallback fails the scenario: passing the oracle comparison on a
# silent host path would not show that the device path works.
_GROUPING = "a GroupBy without an aggregating result selector yields Grouping objects (the group " \
            "as a Python sequence), or its selector builds a Python object from the group"
_USER_AGG = "the aggregate is user Python code (a decomposable class's Seed / Accumulate / " \
            "RecursiveAccumulate)"
_TEXT = "the lambda calls Python str methods on the record (indexing, upper(), split())"
_APPLY = "Apply / ApplyWithPartitionIndex bodies are arbitrary Python over the partition's sequence " \
         "(only @device_function bodies run on HBM tables)"
_OBJECTS = "the records are Python objects with nullable / None / nested fields: no column layout"
_DICT = "the result selector builds a dict / list / nested tuple per record"

ALLOWED_FALLBACKS = {
    "test_empty_inputs": {"group_by": _GROUPING},
    "test_user_types_in_query": {"group_by": _GROUPING},
    "test_DistributiveResultSelector_and_Select": {"group_by": _GROUPING},
    "test_GroupByReduceWithCustomDecomposableFunction_NonDistributableCombiner": {"group_by": _GROUPING},
    "test_GroupByReduce_BitwiseNegationOperator": {"group_by": _GROUPING},
    "test_GroupByWithAnonymousTypes_Pipeline_and_Nested": {"group_by": _GROUPING, "group_partial": _DICT,
                                                          "select": _DICT},
    "test_groupby_decomposable_aggregates": {"group_final": _DICT},
    "test_groupby_with_comparer": {"group_partial": "GroupBy with a user IEqualityComparer (Python Equals)"},
    "test_user_decomposable": {"group_partial": _USER_AGG},
    "test_GroupByReduceWithCustomDecomposableFunction_DistributableCombiner_DifferingTypes_NoFinalizer":
        {"group_partial": _USER_AGG},
    "test_GroupByReduce_BuiltIn_First": {"group_partial": "First depends on the record order inside a group, "
                                                          "which the device grouping kernels do not keep"},
    "test_GroupByReduce_ResultSelector_ComplexNewExpression_and_ListInitializer": {"group_partial": _USER_AGG},
    "test_GroupByReduce_UseAllInternalDecomposables_and_SameDecomposableUsedTwice": {"group_partial": _USER_AGG},
    "test_Aggregate_WithCombiner": {"agg_partial": "Aggregate with a user accumulator / combiner function"},
    "test_groupby_variants": {"group_partial": _TEXT, "hash_partition": _TEXT},
    "test_GroupByReduce_ProgrammingManualExample": {"group_partial": _TEXT},
    "test_selectmany_result_selector": {"select_many": _TEXT},
    "test_hash_partition_overloads": {"apply_index": _APPLY},
    "test_Bug14192_MultiApplySubExpressionReuse": {"apply": _APPLY},
    "test_FullHomomorphicBinaryApply_IdenticalDataSets": {"apply": _APPLY},
    "test_indexed_select_where_selectmany": {"select_many_idx": "indexed SelectMany returning a variable-length Python list"},
    "test_Bug11638_LongMethods": {"select_many_idx": "indexed SelectMany returning a variable-length Python list"},
    "test_Bug13529_and_Bug13593_IndexedOperatorCompilation":
        {"select_many_idx": "indexed SelectMany returning a variable-length Python list"},
    "test_join_and_groupjoin": {"hash_group_join": "GroupJoin result selector iterates the Python group (len(os))"},
    "test_Bug15159_NotOperatorForNullableBool": {"enumerable": _OBJECTS,
                                                 "where": "Python identity comparison (`is None`) on a record"},
    "test_Bug15570_GetHashCodeAndEqualsForNullableFieldsOfAnonymousTypes": {"enumerable": _OBJECTS},
    "test_NonSealedTypeRecords_and_DerivedTypeRecords": {"enumerable": _OBJECTS, "group_partial": _OBJECTS,
                                                         "select": _OBJECTS},
    "test_ObjectRecords": {"enumerable": _OBJECTS},
}

_COVERAGE = collections.Counter()      # (operator, "device" | "host") over every scenario


def _gpu_jobs():
    ctxs = [c for (mode, *_), c in helpers._CTX.items() if mode == "gpu"]
    return [j for c in ctxs for j in c._get_executor().job_log]


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
    for c in [c for (mode, *_), c in helpers._CTX.items() if mode == "gpu"]:
        c._get_executor().job_log.clear()
    fn(**kwargs)
    jobs = _gpu_jobs()
    allowed = ALLOWED_FALLBACKS.get(name, {})
    for j in jobs:
        for k, v in j["op_counts"].items():
            op, where = k.rsplit(":", 1)
            _COVERAGE[(op, where)] += v
    unexplained = sorted({(stage, op, why) for j in jobs for stage, op, why in j["fallbacks"] if op not in allowed})
    assert not unexplained, f"{name}: host fallbacks not in ALLOWED_FALLBACKS: {unexplained}"


def test_zz_print_device_coverage():
    """Per-operator executions on the device vs on the host over the scenarios above."""
    ops = sorted({op for op, _ in _COVERAGE})
    lines = [f"{op:24s} device {_COVERAGE[(op, 'device')]:5d}   host {_COVERAGE[(op, 'host')]:5d}" for op in ops]
    text = "[oracle suites on the GPU executor: operator executions]\n" + "\n".join(lines) + "\n"
    print("\n" + text)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "oracle_device_coverage.txt"), "w") as f:
            f.write(text)
