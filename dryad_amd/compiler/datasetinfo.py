"""Physical data-set properties used to elide shuffles and sorts.

Reference: LinqToDryad/DataSetInfo.cs:91-799 — ``PartitionType {Random, Hash, Range,
HashOrRange}``, ``PartitionInfo`` (IsPartitionedBy / IsSamePartition / CreatePartitionNode),
``OrderByInfo``, ``DistinctInfo``.  Key functions are compared by identity (the reference compares
expression trees structurally with ExpressionMatcher; Python callables are compared by object
identity or by an explicit ``key_name`` given to the operator).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field


class PartitionType(enum.Enum):
    RANDOM = "Random"
    HASH = "Hash"
    RANGE = "Range"
    HASH_OR_RANGE = "HashOrRange"


def same_key(a, b) -> bool:
    if a is None or b is None:
        return False
    if a is b:
        return True
    ka = getattr(a, "_dryad_key_name", None)
    kb = getattr(b, "_dryad_key_name", None)
    if ka is not None and ka == kb:
        return True
    ca, cb = getattr(a, "__code__", None), getattr(b, "__code__", None)
    if ca is not None and cb is not None and ca.co_code == cb.co_code and ca.co_consts == cb.co_consts \
            and ca.co_names == cb.co_names and not getattr(a, "__closure__", None) and not getattr(b, "__closure__", None):
        return True
    return False


@dataclass
class PartitionInfo:
    kind: PartitionType = PartitionType.RANDOM
    count: int = 1
    key: object = None
    comparer: object = None
    separators: list | None = None
    descending: bool = False
    # the range_partition op that produced this partitioning.  A consumer that relies on equal
    # keys being co-located marks it ``keep_ties``; otherwise the GPU executor's fused OrderBy may
    # split long runs of equal keys over several ranks (skew), which keeps the global order but
    # not the co-location.
    origin: dict | None = field(default=None, compare=False, repr=False)
    # sampled range partitions: identity of the separator stage that cut the key space (two data
    # sets range-partitioned by the SAME sampled separators are co-partitioned)
    seps_id: int | None = field(default=None, compare=False, repr=False)

    @staticmethod
    def random(count: int) -> "PartitionInfo":
        return PartitionInfo(PartitionType.RANDOM, count)

    @staticmethod
    def hash(key, count, comparer=None) -> "PartitionInfo":
        return PartitionInfo(PartitionType.HASH, count, key, comparer)

    @staticmethod
    def range(key, count, separators=None, descending=False, comparer=None, origin=None,
              seps_id=None) -> "PartitionInfo":
        return PartitionInfo(PartitionType.RANGE, count, key, comparer, separators, descending, origin, seps_id)

    def rely_on_colocation(self):
        """A consumer elides a shuffle because equal keys share a partition: the producing range
        partition must then keep runs of equal keys together."""
        if self.kind == PartitionType.RANGE and self.origin is not None:
            self.origin["keep_ties"] = True

    def is_partitioned_by(self, key, comparer=None) -> bool:
        """Records with equal keys are guaranteed to be in the same partition (a True answer
        marks the producing range partition keep_ties, see ``origin``)."""
        if self.count == 1:
            return True
        if self.kind in (PartitionType.HASH, PartitionType.RANGE, PartitionType.HASH_OR_RANGE):
            ok = same_key(self.key, key) and (comparer is None or comparer is self.comparer)
            if ok:
                self.rely_on_colocation()
            return ok
        return False

    def is_same_partition(self, other: "PartitionInfo") -> bool:
        """Two data sets are co-partitioned (equal keys land in equal partition indexes)."""
        if self.count != other.count:
            return False
        if self.count == 1:
            return True
        if self.kind == PartitionType.HASH and other.kind == PartitionType.HASH:
            return True   # same hash function and count; keys compared by the caller
        if self.kind == PartitionType.RANGE and other.kind == PartitionType.RANGE:
            same = (self.separators is not None and self.separators == other.separators) or (
                self.seps_id is not None and self.seps_id == other.seps_id)
            ok = same and self.descending == other.descending
            if ok:
                self.rely_on_colocation()
                other.rely_on_colocation()
            return ok
        return False


@dataclass
class OrderInfo:
    key: object = None
    comparer: object = None
    descending: bool = False

    def is_ordered_by(self, key, comparer=None, descending=False) -> bool:
        return self.key is not None and same_key(self.key, key) and self.descending == descending and (
            comparer is None or comparer is self.comparer)


@dataclass
class DataSetInfo:
    partition: PartitionInfo = field(default_factory=lambda: PartitionInfo.random(1))
    order: OrderInfo | None = None           # order *within* each partition
    distinct: bool = False
    partition_ordered: bool = True           # the partitions' concatenation preserves the query order

    def with_count(self, n: int) -> "DataSetInfo":
        return DataSetInfo(PartitionInfo.random(n), None, False, True)

    def describe(self) -> str:
        p = self.partition
        s = f"{p.kind.value}({p.count})"
        if self.order is not None:
            s += " ordered" + (" desc" if self.order.descending else "")
        if self.distinct:
            s += " distinct"
        return s
