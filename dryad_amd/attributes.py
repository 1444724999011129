"""User extensibility attributes (reference LinqToDryad/Attributes.cs:37-445, IDecomposable.cs,
IAssociative.cs) as Python decorators and protocols.

* ``@homomorphic`` / ``@homomorphic(left=True)`` — an Apply function that distributes over
  partitions (reference ``[Homomorphic]``), so Apply runs per partition without merging.
* ``@resource(is_stateful=..., is_expensive=...)`` — ``[Resource]``: expensive functions are never
  duplicated by pipeline fusion; stateful ones force sequential evaluation.
* ``@decomposable(DecomposerClass)`` — ``[Decomposable(typeof(IDecomposable<S,A,R>))]``: marks an
  aggregate function used inside a GroupBy result selector as decomposable into
  Initialize/Seed/Accumulate/RecursiveAccumulate/FinalReduce (combiner inference, §E-4).
* ``@associative(AssociativeClass)`` — ``[Associative(typeof(IAssociative<A>))]``: Seed +
  RecursiveAccumulate; Aggregate with such a function is computed as a tree.
* ``@nullable`` on a dataclass field type via ``typing.Optional`` (the ``[Nullable]`` attribute).
* ``@custom_serializer(cls)`` — ``[CustomDryadLinqSerializer]``: the class provides
  ``Write(writer, value)`` / ``Read(reader)``.
* ``@device_function`` — (no reference equivalent: the reference's vertex code is CLR) an
  Apply/ApplyPerPartition body that takes and returns ``gpu.table.DeviceTable`` partitions.  On
  the GPU executor it runs on the HBM-resident tensors (HIP kernels / torch); LocalDebug and the
  CPU executors hand it CPU-tensor tables built from the records, so one body serves every
  executor.
"""
from __future__ import annotations

import functools


class IDecomposable:
    """Protocol: Initialize(state); Seed(x) -> acc; Accumulate(acc, x) -> acc;
    RecursiveAccumulate(acc, acc) -> acc; FinalReduce(acc) -> result."""

    def Initialize(self, state):
        pass

    def Seed(self, x):  # pragma: no cover - protocol
        raise NotImplementedError

    def Accumulate(self, acc, x):  # pragma: no cover
        raise NotImplementedError

    def RecursiveAccumulate(self, a, b):  # pragma: no cover
        raise NotImplementedError

    def FinalReduce(self, acc):  # pragma: no cover
        raise NotImplementedError


class IAssociative:
    """Protocol: Seed() -> acc; RecursiveAccumulate(acc, acc) -> acc."""

    def Seed(self):  # pragma: no cover
        raise NotImplementedError

    def RecursiveAccumulate(self, a, b):  # pragma: no cover
        raise NotImplementedError


def _mark(fn, **attrs):
    for k, v in attrs.items():
        setattr(fn, k, v)
    return fn


def homomorphic(fn=None, *, left=False):
    def deco(f):
        return _mark(f, _dryad_homomorphic=True, _dryad_left_homomorphic=bool(left))
    return deco(fn) if fn is not None else deco


def resource(is_stateful: bool = False, is_expensive: bool = False):
    def deco(f):
        return _mark(f, _dryad_stateful=is_stateful, _dryad_expensive=is_expensive)
    return deco


def decomposable(decomposer_cls):
    if not all(hasattr(decomposer_cls, m) for m in ("Seed", "Accumulate", "RecursiveAccumulate", "FinalReduce")):
        from .errors import DryadLinqException, ErrorCode
        raise DryadLinqException(ErrorCode.DecomposerTypeDoesNotImplementInterface,
                                 f"{decomposer_cls.__name__} does not implement IDecomposable")

    def deco(f):
        @functools.wraps(f)
        def w(group, *a, **k):
            from .compiler.decomposition import user_decomposable_call
            return user_decomposable_call(f, decomposer_cls, group, a)
        return _mark(w, _dryad_decomposable=decomposer_cls)
    return deco


def associative(assoc_cls):
    def deco(f):
        @functools.wraps(f)
        def w(*a, **k):
            return f(*a, **k)
        return _mark(w, _dryad_associative=assoc_cls)
    return deco


def custom_serializer(serializer_cls):
    def deco(cls):
        cls._dryad_serializer = serializer_cls
        return cls
    return deco


def device_function(fn):
    """Mark an Apply body as a DeviceTable -> DeviceTable function (see module docstring)."""
    return _mark(fn, _dryad_device=True)


def is_device_function(f) -> bool:
    return bool(getattr(f, "_dryad_device", False))


def is_homomorphic(f) -> bool:
    return bool(getattr(f, "_dryad_homomorphic", False))


def is_left_homomorphic(f) -> bool:
    return bool(getattr(f, "_dryad_left_homomorphic", False))


def is_expensive(f) -> bool:
    return bool(getattr(f, "_dryad_expensive", False))


def is_stateful(f) -> bool:
    return bool(getattr(f, "_dryad_stateful", False))
