"""Combiner inference for GroupBy result selectors (decomposable aggregates).

Reference: LinqToDryad/DryadLinqDecomposition.cs:81-922 — recognises Count/LongCount/Any/All/
First/Last/Sum/Min/Max/Aggregate/Average/Contains/Distinct and user ``[Decomposable]`` /
``[Associative]`` functions inside a GroupBy result selector and rewrites the GroupBy into a local
partial aggregation (Seed/Accumulate) + shuffle + final aggregation (RecursiveAccumulate /
FinalReduce) — the classic map-side combiner.

C# result selectors are expression trees; Python lambdas are opaque, so the selector is traced
once, symbolically: it is called with a ``Sym`` key and a ``GroupProxy`` whose LINQ-style methods
(``g.Count()``, ``g.Sum(f)``, ...) return ``Sym`` aggregate placeholders.  The returned structure
(tuple / list / dict / dataclass / namedtuple / scalar, possibly arithmetic on placeholders) is the
*template*; at run time each group's aggregate values are substituted into it.  Anything the tracer
cannot see through (iterating the group, ``len(g)``, branching on a placeholder) makes the selector
non-decomposable and the planner falls back to a full shuffle + GroupBy.
"""
from __future__ import annotations

import dataclasses
import operator

from ..attributes import IDecomposable


class NotDecomposable(Exception):
    pass


# ---------------------------------------------------------------------------------------------
class Sym:
    """Symbolic value recorded while tracing a result selector."""
    __slots__ = ("fn", "args")

    def __init__(self, fn, args):
        object.__setattr__(self, "fn", fn)
        object.__setattr__(self, "args", args)

    def eval(self, env):
        if self.fn == "key":
            return env["key"]
        if self.fn == "agg":
            return env["aggs"][self.args[0]]
        if self.fn == "const":
            return self.args[0]
        vals = [a.eval(env) if isinstance(a, Sym) else a for a in self.args]
        if self.fn == "getattr":
            return getattr(vals[0], vals[1])
        if self.fn == "getitem":
            return vals[0][vals[1]]
        if self.fn == "call":
            f, *rest = vals
            return f(*rest)
        if self.fn == "method":
            obj, name, *rest = vals
            return getattr(obj, name)(*rest)
        return self.fn(*vals)

    # attribute / item access on keys (e.g. g.Key.Name, g.Key[0])
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return Sym("getattr", (self, name))

    def __getitem__(self, k):
        return Sym("getitem", (self, k))

    def __call__(self, *a):
        return Sym("call", (self,) + a)

    def __bool__(self):
        raise NotDecomposable("branch on an aggregate value")

    def __len__(self):
        raise NotDecomposable("len() of a symbolic value")

    def __iter__(self):
        raise NotDecomposable("iteration of a symbolic value")

    def __hash__(self):
        return id(self)

    def __str__(self):
        raise NotDecomposable("str() of a symbolic value")

    def __format__(self, spec):
        raise NotDecomposable("format() of a symbolic value")

    def __index__(self):
        raise NotDecomposable("index use of a symbolic value")

    def __repr__(self):
        return f"Sym({self.fn!r})"


def _binop(fn):
    return lambda self, o: Sym(fn, (self, o))


def _rbinop(fn):
    return lambda self, o: Sym(lambda a, b: fn(b, a), (self, o))


for _n, _f in [("add", operator.add), ("sub", operator.sub), ("mul", operator.mul), ("truediv", operator.truediv),
               ("floordiv", operator.floordiv), ("mod", operator.mod), ("pow", operator.pow),
               ("and", operator.and_), ("or", operator.or_), ("xor", operator.xor),
               ("lt", operator.lt), ("le", operator.le), ("gt", operator.gt), ("ge", operator.ge),
               ("eq", operator.eq), ("ne", operator.ne)]:
    setattr(Sym, f"__{_n}__", _binop(_f))
    if _n not in ("lt", "le", "gt", "ge", "eq", "ne"):
        setattr(Sym, f"__r{_n}__", _rbinop(_f))
Sym.__neg__ = lambda self: Sym(operator.neg, (self,))
Sym.__abs__ = lambda self: Sym(abs, (self,))
Sym.__float__ = lambda self: (_ for _ in ()).throw(NotDecomposable("float() of symbolic value"))
Sym.__int__ = lambda self: (_ for _ in ()).throw(NotDecomposable("int() of symbolic value"))
Sym.__round__ = lambda self, nd=None: Sym(round, (self,) if nd is None else (self, nd))


# ---------------------------------------------------------------------------------------------
# Aggregate kinds.  Each is (seed(x), accumulate(acc, x), combine(acc, acc), final(acc)).
class _MissingType:
    """Picklable singleton (accumulators cross process boundaries in channels)."""

    def __reduce__(self):
        return "_MISSING"

    def __repr__(self):
        return "<missing>"


_MISSING = _MissingType()


class Agg:
    def __init__(self, kind, sel=None, pred=None, extra=None):
        self.kind, self.sel, self.pred, self.extra = kind, sel, pred, extra

    def _v(self, x):
        return self.sel(x) if self.sel is not None else x

    def seed(self, x):
        k = self.kind
        if k == "count":
            return 1 if (self.pred is None or self.pred(x)) else 0
        if k == "sum":
            v = self._v(x)
            return 0 if v is None else v
        if k in ("min", "max"):
            v = self._v(x)
            return _MISSING if v is None else v
        if k == "avg":
            v = self._v(x)
            return (0, 0) if v is None else (v, 1)
        if k == "any":
            return bool(self.pred(x)) if self.pred is not None else True
        if k == "all":
            return bool(self.pred(x))
        if k == "contains":
            return x == self.extra
        if k == "first":
            return x if self.pred is None or self.pred(x) else _MISSING
        if k == "last":
            return x if self.pred is None or self.pred(x) else _MISSING
        if k == "distinct":
            return {self._v(x)}
        if k == "user":
            return self.extra.Seed(x)
        if k == "assoc":
            return self.extra.RecursiveAccumulate(self.extra.Seed(), self._v(x)) if hasattr(self.extra, "Seed") \
                else self._v(x)
        raise NotDecomposable(k)

    def accumulate(self, acc, x):
        k = self.kind
        if k == "user":
            return self.extra.Accumulate(acc, x)
        return self.combine(acc, self.seed(x))

    def combine(self, a, b):
        k = self.kind
        if k in ("count", "sum"):
            return a + b
        if k == "min":
            return b if a is _MISSING else a if b is _MISSING else (b if b < a else a)
        if k == "max":
            return b if a is _MISSING else a if b is _MISSING else (b if b > a else a)
        if k == "avg":
            return (a[0] + b[0], a[1] + b[1])
        if k in ("any", "contains"):
            return a or b
        if k == "all":
            return a and b
        if k == "first":
            return a if a is not _MISSING else b
        if k == "last":
            return b if b is not _MISSING else a
        if k == "distinct":
            return a | b
        if k == "user":
            return self.extra.RecursiveAccumulate(a, b)
        if k == "assoc":
            return self.extra.RecursiveAccumulate(a, b)
        raise NotDecomposable(k)

    def final(self, acc):
        k = self.kind
        if k in ("min", "max", "first", "last") and acc is _MISSING:
            from ..enumerable import InvalidOperationException
            raise InvalidOperationException("Sequence contains no elements")
        if k == "avg":
            if acc[1] == 0:
                from ..enumerable import InvalidOperationException
                raise InvalidOperationException("Sequence contains no elements")
            return acc[0] / acc[1]
        if k == "distinct":
            return sorted(acc, key=repr)
        if k == "user":
            return self.extra.FinalReduce(acc)
        return acc


class GroupProxy:
    """Stands in for the IGrouping while tracing; records aggregate calls."""

    def __init__(self, aggs: list):
        self._aggs = aggs
        self.Key = Sym("key", ())

    def _add(self, agg):
        self._aggs.append(agg)
        return Sym("agg", (len(self._aggs) - 1,))

    def Count(self, predicate=None):
        return self._add(Agg("count", pred=predicate))

    LongCount = Count

    def Sum(self, selector=None):
        return self._add(Agg("sum", sel=selector))

    def Min(self, selector=None):
        return self._add(Agg("min", sel=selector))

    def Max(self, selector=None):
        return self._add(Agg("max", sel=selector))

    def Average(self, selector=None):
        return self._add(Agg("avg", sel=selector))

    def Any(self, predicate=None):
        return self._add(Agg("any", pred=predicate))

    def All(self, predicate):
        return self._add(Agg("all", pred=predicate))

    def Contains(self, value):
        return self._add(Agg("contains", extra=value))

    def First(self, predicate=None):
        return self._add(Agg("first", pred=predicate))

    def Last(self, predicate=None):
        return self._add(Agg("last", pred=predicate))

    def Distinct(self, selector=None):
        return self._add(Agg("distinct", sel=selector))

    def Aggregate(self, *args):
        # only associative aggregations decompose: Aggregate(func) with an @associative func
        func = args[-1] if args else None
        assoc = getattr(func, "_dryad_associative", None)
        if assoc is None:
            raise NotDecomposable("Aggregate without an [Associative] function")
        return self._add(Agg("assoc", extra=assoc()))

    def Select(self, *a):
        raise NotDecomposable("Select over a group")

    def __iter__(self):
        raise NotDecomposable("iterating the group")

    def __len__(self):
        raise NotDecomposable("len(group) (use g.Count())")

    def apply_user(self, decomposer_cls, selector=None):
        d = decomposer_cls()
        if hasattr(d, "Initialize"):
            d.Initialize(None)
        return self._add(Agg("user", sel=selector, extra=d))


@dataclasses.dataclass
class Decomposition:
    aggs: list
    template: object

    def seed(self, x):
        return [a.seed(x) for a in self.aggs]

    def accumulate(self, accs, x):
        return [a.accumulate(s, x) for a, s in zip(self.aggs, accs)]

    def combine(self, a, b):
        return [ag.combine(x, y) for ag, x, y in zip(self.aggs, a, b)]

    def final(self, key, accs):
        vals = [a.final(s) for a, s in zip(self.aggs, accs)]
        return substitute(self.template, {"key": key, "aggs": vals})


def substitute(t, env):
    if isinstance(t, Sym):
        return t.eval(env)
    if isinstance(t, tuple):
        if hasattr(t, "_fields"):
            return type(t)(*[substitute(x, env) for x in t])
        return tuple(substitute(x, env) for x in t)
    if isinstance(t, list):
        return [substitute(x, env) for x in t]
    if isinstance(t, dict):
        return {substitute(k, env): substitute(v, env) for k, v in t.items()}
    if dataclasses.is_dataclass(t) and not isinstance(t, type):
        return type(t)(**{f.name: substitute(getattr(t, f.name), env) for f in dataclasses.fields(t)})
    return t


def _contains_sym(t) -> bool:
    if isinstance(t, Sym):
        return True
    if isinstance(t, (tuple, list)):
        return any(_contains_sym(x) for x in t)
    if isinstance(t, dict):
        return any(_contains_sym(k) or _contains_sym(v) for k, v in t.items())
    if dataclasses.is_dataclass(t) and not isinstance(t, type):
        return any(_contains_sym(getattr(t, f.name)) for f in dataclasses.fields(t))
    return False


def decompose(result_selector, element_selector=None) -> Decomposition | None:
    """Try to decompose ``result_selector(key, group)``; None if not decomposable."""
    if result_selector is None:
        return None
    from ..gpu.trace import uses_identity
    if uses_identity(result_selector) or (element_selector is not None and uses_identity(element_selector)):
        return None             # `is` on a symbolic key / group cannot be decided per group
    aggs: list = []
    g = GroupProxy(aggs)
    try:
        tmpl = result_selector(g.Key, g)
    except NotDecomposable:
        return None
    except Exception:
        return None
    if not aggs:
        return None
    if element_selector is not None:
        # aggregate selectors see projected elements
        for a in aggs:
            inner_sel, inner_pred = a.sel, a.pred
            es = element_selector
            if inner_sel is not None:
                a.sel = (lambda s, e: lambda x: s(e(x)))(inner_sel, es)
            elif a.kind not in ("count",):
                a.sel = es
            if inner_pred is not None:
                a.pred = (lambda p, e: lambda x: p(e(x)))(inner_pred, es)
            if a.kind == "user":
                d = a.extra
                a.kind = "user"
                a.extra = _ProjectedDecomposer(d, es)
    return Decomposition(aggs, tmpl)


class _ProjectedDecomposer(IDecomposable):
    def __init__(self, d, sel):
        self.d, self.sel = d, sel

    def Seed(self, x):
        return self.d.Seed(self.sel(x))

    def Accumulate(self, a, x):
        return self.d.Accumulate(a, self.sel(x))

    def RecursiveAccumulate(self, a, b):
        return self.d.RecursiveAccumulate(a, b)

    def FinalReduce(self, a):
        return self.d.FinalReduce(a)


def user_decomposable_call(fn, decomposer_cls, group, args):
    """Hook used by @decomposable wrappers: when called on a GroupProxy while tracing, record a
    user aggregate instead of running the function."""
    if isinstance(group, GroupProxy):
        sel = args[0] if args else None
        return group.apply_user(decomposer_cls, sel)
    return fn(group, *args)
