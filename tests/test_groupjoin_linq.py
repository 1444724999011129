"""GroupJoin hands the result selector an IEnumerable-like group (g.Count(), g.Sum(...) work, as
on IEnumerable<TInner> in the reference) in LocalDebug and on the process executor; the GPU
executor's device GroupJoin relies on the same spelling."""
from helpers import both


def test_group_join_group_has_linq_methods():
    outer = list(range(20))
    inner = [i % 7 for i in range(50)]
    r = both(lambda c: c.FromEnumerable(outer).GroupJoin(
        c.FromEnumerable(inner), lambda x: x, lambda y: y,
        lambda x, g: (x, g.Count(), len(g), g.Sum(lambda y: y * 2))))
    exp = [(x, sum(1 for y in inner if y == x), sum(1 for y in inner if y == x), sum(2 * y for y in inner if y == x))
           for x in outer]
    assert sorted(r) == sorted(exp)
