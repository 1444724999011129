"""Expression-level rewrites applied to fixpoint before planning.

Reference: LinqToDryad/SimpleRewriter.cs:211-327 — push a non-indexed ``Where`` below
``OrderBy``/``Distinct``/``RangePartition``/``HashPartition`` (filter before moving or sorting
data) and distribute ``Where`` over ``Concat``.
"""
from __future__ import annotations

from ..query import QNode

_PUSH_THROUGH = {"OrderBy", "Distinct", "RangePartition", "HashPartition"}


def _clone(n: QNode, sources) -> QNode:
    m = QNode(n.op, sources, dict(n.args), n.dtype, n.port)
    return m


def rewrite(root: QNode) -> QNode:
    memo = {}

    def go(n: QNode) -> QNode:
        if n.id in memo:
            return memo[n.id]
        srcs = [go(s) for s in n.sources]
        out = n if all(a is b for a, b in zip(srcs, n.sources)) else _clone(n, srcs)
        changed = True
        while changed:
            changed = False
            if out.op == "Where" and not out.args.get("indexed") and out.sources:
                child = out.sources[0]
                if child.op in _PUSH_THROUGH and not (child.op == "HashPartition" and child.args.get("result_selector")):
                    # Where(X(c)) -> X(Where(c))
                    inner = QNode("Where", [child.sources[0]], dict(out.args), child.sources[0].dtype)
                    new = QNode(child.op, [inner] + list(child.sources[1:]), dict(child.args), child.dtype, child.port)
                    out = new
                    out_inner = go_rewritten(inner)
                    out = QNode(out.op, [out_inner] + list(out.sources[1:]), dict(out.args), out.dtype, out.port)
                    changed = True
                elif child.op == "Concat":
                    a = go_rewritten(QNode("Where", [child.sources[0]], dict(out.args), child.sources[0].dtype))
                    b = go_rewritten(QNode("Where", [child.sources[1]], dict(out.args), child.sources[1].dtype))
                    out = QNode("Concat", [a, b], dict(child.args), child.dtype)
                    changed = True
        memo[n.id] = out
        return out

    def go_rewritten(n: QNode) -> QNode:
        # sources are already rewritten; re-apply the local rule to the new node
        return go(n)

    return go(root)
