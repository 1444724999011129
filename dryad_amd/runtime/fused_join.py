"""Fused grace / radix hash join for ``outer.Join(inner, ok, ik, result)`` folded by a decomposable
aggregate (Sum / Count / LongCount / Average) — the physical strategy the GPU executor picks for the
plan idiom

    read(outer) -> HashPartition -(cross)-> Merge --.
                                                    +-> Join [+ Select] + agg_partial -> agg_final
    read(inner) -> HashPartition -(cross)-> Merge --'

The reference runs this as HashPartition vertices, N x M file channels, and a ParallelHashJoin vertex
per partition building a hash table over the inner side (DryadLinqQueryGen.VisitJoin
:1419-1609, DryadLinqVertex.HashJoin :852-897 / ParallelHashJoin :6703), with the aggregate as a
separate pipelined operator.  Here the whole idiom is ONE gang stage over ops/grace.GraceHashJoin:

  * column pruning from the traced selectors: the key selectors and the (result selector o Select o
    aggregate selector) composition are traced symbolically to ``a * outer.f + b * inner.g + c``;
    only the key and those two 8-byte fields travel (a byte projection of each row inside the first
    partitioning pass, or a [key, value] row per side when the two layouts differ);
  * both inputs are read chunk by chunk (gen://records64 generated in place, hbm:// column tables
    packed), hash-routed to their rank over xGMI (RCCL all-to-all-v) and into hash buckets that stay
    in HBM while the budget (``HbmBudgetBytes``) allows, the rest spilling to pinned host DRAM;
  * every bucket pair is joined with the aggregate fused into the probe (matches, sum of the build
    field, sum of the probe field): the LDS radix join when all buckets are resident, the global
    hash table bucket by bucket otherwise.

The stage's output is exactly what ``agg_partial`` would have produced for each partition, so the
final aggregate vertex is unchanged.  Sums are 64-bit integer sums of int64 fields.
"""
from __future__ import annotations

import torch

from ..gpu.table import DeviceTable
from ..io.providers import GenProvider, parse_uri, provider_for
from ..parallel import shuffle
from ..utils.log import get_logger

log = get_logger("fused_join")

AGG_KINDS = ("Sum", "Count", "LongCount", "Average")
CHUNK_ROWS = 1 << 27


# ------------------------------------------------------------------------------------------------
# symbolic linear tracing
class NotLinear(Exception):
    pass


class Lin:
    """``sum(coef * field) + const`` over (side, field index) terms, integer coefficients."""

    def __init__(self, terms=None, const=0):
        self.terms = {k: v for k, v in (terms or {}).items() if v}
        self.const = const

    @staticmethod
    def of(x):
        if isinstance(x, Lin):
            return x
        if isinstance(x, bool) or not isinstance(x, int):
            raise NotLinear(f"non-integer constant {x!r}")
        return Lin(None, x)

    def __add__(self, o):
        o = Lin.of(o)
        t = dict(self.terms)
        for k, v in o.terms.items():
            t[k] = t.get(k, 0) + v
        return Lin(t, self.const + o.const)

    __radd__ = __add__

    def __neg__(self):
        return Lin({k: -v for k, v in self.terms.items()}, -self.const)

    def __sub__(self, o):
        return self + (-Lin.of(o))

    def __rsub__(self, o):
        return Lin.of(o) + (-self)

    def __mul__(self, o):
        o = Lin.of(o)
        if o.terms and self.terms:
            raise NotLinear("product of two fields")
        if o.terms:
            return o * self.const
        return Lin({k: v * o.const for k, v in self.terms.items()}, self.const * o.const)

    __rmul__ = __mul__

    def __pos__(self):
        return self

    def __bool__(self):
        raise NotLinear("truth value of a field")

    def __getattr__(self, name):
        raise NotLinear(f"attribute {name} of a field")


class _Rec:
    def __init__(self, side, fields):
        self._side, self._fields = side, list(fields)

    def __getitem__(self, i):
        if isinstance(i, bool) or not isinstance(i, int) or not -len(self._fields) <= i < len(self._fields):
            raise NotLinear(f"record index {i!r}")
        return Lin({(self._side, i % len(self._fields)): 1})

    def __getattr__(self, name):
        if name.startswith("_") or name not in self._fields:
            raise NotLinear(f"record field {name}")
        return Lin({(self._side, self._fields.index(name)): 1})


def _trace(fn, *args) -> Lin:
    try:
        r = fn(*args)
    except NotLinear:
        raise
    except Exception as e:  # noqa: BLE001
        raise NotLinear(f"{type(e).__name__}: {e}") from e
    return Lin.of(r)


def _key_field(fn, side, fields) -> int:
    k = _trace(fn, _Rec(side, fields))
    if k.const or len(k.terms) != 1 or next(iter(k.terms.values())) != 1:
        raise NotLinear("key is not a single field")
    return next(iter(k.terms))[1]


# ------------------------------------------------------------------------------------------------
# plan idiom
def find(plan) -> dict:
    """{join stage id: descriptor} for every fusable Join + aggregate idiom of the plan.  Each
    join input is either a read stage feeding the join pointwise (one partition per side), or
    read + HashPartition -(cross)-> Merge; the join stage's program is join [select...]
    agg_partial [anything after: run on the fused output]."""
    st = plan.stages
    out = {}
    for j in st:
        ops = [o["op"] for o in j.ops]
        if not ops or ops[0] not in ("hash_join", "merge_join") or "agg_partial" not in ops:
            continue
        k = ops.index("agg_partial")
        if any(o != "select" for o in ops[1:k]) or j.ops[k]["spec"].get("kind") not in AGG_KINDS:
            continue
        if j.ops[k]["spec"].get("predicate") is not None or j.ops[0].get("comparer") is not None:
            continue
        if len(j.inputs) != 2:
            continue
        sides = []
        for inp in j.inputs:
            m = st[inp.src]
            if inp.kind == "cross":           # Merge vertex elided by the planner's cleanup
                if [o["op"] for o in m.ops] != ["read", "hash_partition"] or m.inputs or \
                        plan.consumers(m.id) != [j.id]:
                    break
                sides.append((m, None))
                continue
            if inp.kind != "pointwise":
                break
            if [o["op"] for o in m.ops] == ["read"] and not m.inputs and plan.consumers(m.id) == [j.id] \
                    and not m.is_output:
                sides.append((m, None))
                continue
            if [o["op"] for o in m.ops] != ["identity"] or len(m.inputs) != 1 or m.inputs[0].kind != "cross":
                break
            hp = st[m.inputs[0].src]
            if [o["op"] for o in hp.ops] != ["read", "hash_partition"] or hp.inputs:
                break
            if plan.consumers(hp.id) != [m.id] or plan.consumers(m.id) != [j.id]:
                break
            sides.append((hp, m))
        if len(sides) != 2 or sides[0][0].id == sides[1][0].id:
            continue
        if len({j.partitions} | {x.partitions for sd in sides for x in sd if x is not None}) != 1:
            continue
        stages = [x.id for sd in sides for x in sd if x is not None]
        out[j.id] = dict(join=j.id, stages=stages, reads=[sides[0][0].ops[0], sides[1][0].ops[0]], op=j.ops[0],
                         selects=j.ops[1:k], agg=j.ops[k]["spec"], rest=j.ops[k + 1:])
    return out


# ------------------------------------------------------------------------------------------------
# row sources
class _GenRows:
    """gen://records64 partition rows generated chunk by chunk ([c, ncols] int64 = 8 * ncols B)."""

    def __init__(self, uri, part):
        _, _, q = parse_uri(uri)
        self.lo, self.hi = GenProvider().bounds(uri, part)
        self.n = self.hi - self.lo
        self.ncols = int(q.get("cols", 8))
        from ..models.records_cpu import FIELDS, dim_multiplier
        self.fields = FIELDS[: self.ncols]
        self.dtypes = [torch.int64] * self.ncols
        self.nk = int(q.get("keys", 1 << 20))
        self.seed = int(q.get("seed", 0))
        self.dim = dim_multiplier(self.nk) if q.get("mode") == "dim" else 0
        self.buf = None

    def chunk(self, a, b, dev):
        from ..ops import relational as R
        if self.buf is None or self.buf.numel() < (b - a) * self.ncols:
            self.buf = torch.empty(max(b - a, 1) * self.ncols, dtype=torch.int64, device=dev)
        rows = self.buf[: (b - a) * self.ncols].view(b - a, self.ncols)
        if b > a:
            R.gen_records64_rows(rows, self.lo + a, self.nk, self.seed, self.dim)
        return rows


class _TableRows:
    """A resident columnar partition (hbm://): chunks of its int64 columns stacked into rows."""

    def __init__(self, table: DeviceTable):
        self.t = table
        self.n = table.n
        self.fields = list(table.shape.fields)
        self.dtypes = [table.cols[f].dtype if f in table.cols and table.cols[f].dim() == 1 else None
                       for f in self.fields]

    def chunk(self, a, b, dev):
        return torch.stack([self.t.cols[f][a:b] for f in self.fields], 1) if b > a else \
            torch.empty((0, len(self.fields)), dtype=torch.int64, device=dev)


def _source(read_op, part):
    scheme, path, q = parse_uri(read_op["uri"])
    if scheme == "gen" and path.strip("/") == "records64":
        return _GenRows(read_op["uri"], part)
    if scheme == "hbm":
        ent = provider_for(read_op["uri"]).get(read_op["uri"])
        t = ent["local"].get(part)
        if isinstance(t, DeviceTable) and t.rows is None and not t.strs and t.heap is None and \
                t.shape.kind in ("tuple", "dataclass") and t.cols:
            return _TableRows(t)
    return None


# ------------------------------------------------------------------------------------------------
def _local_parts(desc, runner) -> list:
    P, W, me = runner.plan.stages[desc["join"]].partitions, runner.world.size, runner.world.rank
    return [p for p in range(P) if runner.owner(p) == me]


def plan_local(desc, runner):
    """This rank's half of the applicability vote: (ok, layout) where layout describes the fields
    to keep.  Every rank must agree (the caller all-gathers the votes)."""
    if not runner.gpu_ok:
        return None
    parts = _local_parts(desc, runner)
    srcs = [[_source(r, p) for p in parts] for r in desc["reads"]]
    if not parts or any(x is None for side in srcs for x in side):
        return None
    if any(len({(tuple(x.fields), tuple(map(str, x.dtypes))) for x in side}) != 1 for side in srcs):
        return None
    srcs = [side[0] for side in srcs]
    fo, fi = srcs[0].fields, srcs[1].fields
    op = desc["op"]
    try:
        ko = _key_field(op["outer_key"], 0, fo)
        ki = _key_field(op["inner_key"], 1, fi)
        val = _trace(op["result"], _Rec(0, fo), _Rec(1, fi))
        for s in desc["selects"]:
            val = _trace(s["fn"], val)
        agg = desc["agg"]
        if agg["kind"] in ("Sum", "Average") and agg.get("selector") is not None:
            val = _trace(agg["selector"], val)
    except NotLinear as e:
        log.info("join %s not fused: %s", desc["join"], e)
        return None
    if agg["kind"] in ("Count", "LongCount"):
        val = Lin(None, 0)
    per_side = [[(f, c) for (sd, f), c in val.terms.items() if sd == side] for side in (0, 1)]
    if any(len(x) > 1 for x in per_side):
        return None
    need = [srcs[0].dtypes[ko], srcs[1].dtypes[ki]] + [srcs[s].dtypes[f] for s in (0, 1) for f, _ in per_side[s]]
    if any(d != torch.int64 for d in need):
        return None
    vo = per_side[0][0] if per_side[0] else (None, 0)
    vi = per_side[1][0] if per_side[1] else (None, 0)
    return dict(ko=ko, ki=ki, vo=vo[0], co=vo[1], vi=vi[0], ci=vi[1], const=val.const,
                ncols=(len(fo), len(fi)), gen=all(isinstance(s, _GenRows) for s in srcs))


def _layout(lay):
    """Row layout shared by both sides: a byte projection of the source rows when the key and the
    value fields sit at the same place in both tables, else [key, value] rows built per chunk."""
    ko, ki, vo, vi = lay["ko"], lay["ki"], lay["vo"], lay["vi"]
    if lay["gen"] and ko == ki and lay["ncols"][0] == lay["ncols"][1]:
        fields = {ko} | ({vo} if vo is not None else set()) | ({vi} if vi is not None else set())
        lo, hi = min(fields), max(fields) + 1
        if hi - lo == 1:
            hi = lo + 2 if lo + 2 <= lay["ncols"][0] else hi
            lo = hi - 2
        if hi - lo == 2:                  # 16-byte rows: what the LDS radix join takes
            col = lambda f: 8 * (f - lo) if f is not None else 8 * (ko - lo)  # noqa: E731
            return dict(direct=True, proj=(8 * lo, 8 * (hi - lo)), key_off=8 * ko, col_o=col(vo), col_i=col(vi),
                        stride_in=8 * lay["ncols"][0])
    return dict(direct=False, proj=None, key_off=0, col_o=8, col_i=8, stride_in=16)


SAMPLE_KEYS = 1 << 16


def _choose_build(srcs, lay, n_tot, w, dev) -> int:
    """Build side of the bucket hash tables: the smaller input, unless the two are within 2x of
    each other; then the one whose keys repeat less in a sample of each side's first rows (a
    unique-key dimension table beats a fact table with Poisson-repeated keys as the build side)."""
    if max(n_tot) > 2 * max(1, min(n_tot)):
        return 0 if n_tot[0] < n_tot[1] else 1
    ratio = torch.zeros(2, dtype=torch.float64, device=dev)
    for side in (0, 1):
        s = next((x for x in srcs[side] if x.n), None)
        if s is None:
            continue
        m = min(s.n, SAMPLE_KEYS)
        kf = lay["ko"] if side == 0 else lay["ki"]
        keys = s.chunk(0, m, dev)[:, kf]
        ratio[side] = torch.unique(keys).numel() / m
    shuffle.all_reduce_(ratio, "sum", w)
    r = ratio.tolist()
    if abs(r[0] - r[1]) > 0.02:
        return 0 if r[0] > r[1] else 1
    return 0 if n_tot[0] <= n_tot[1] else 1


def run(desc, runner, lay) -> dict:
    """Execute the fused join on this rank -> {local Join partition: its agg_partial output}."""
    from ..ops import grace as GR
    w = runner.world
    W, dev = w.size, runner.dev
    parts = _local_parts(desc, runner)
    srcs = [[_source(r, p) for p in parts] for r in desc["reads"]]
    L = _layout(lay)
    n_loc = torch.tensor([sum(x.n for x in srcs[0]), sum(x.n for x in srcs[1])], dtype=torch.int64, device=dev)
    n_tot, n_max = n_loc.clone(), n_loc.clone()
    shuffle.all_reduce_(n_tot, "sum", w)
    shuffle.all_reduce_(n_max, "max", w)
    n_tot, n_max = n_tot.tolist(), n_max.tolist()
    build = _choose_build(srcs, lay, n_tot, w, dev)
    names = ("O", "I")
    chunk_rows = max(1, min(CHUNK_ROWS, max(n_max)))
    gens = [x for side in srcs for x in side if isinstance(x, _GenRows)]
    if gens:                              # one chunk buffer shared by every generated source
        flat = torch.empty(chunk_rows * max(x.ncols for x in gens), dtype=torch.int64, device=dev)
        for x in gens:
            x.buf = flat
    # chunk schedule per side: the same number of (collective) add_chunk calls on every rank
    sched = []
    for side in (0, 1):
        lst = [(x, a, min(x.n, a + chunk_rows)) for x in srcs[side] for a in range(0, x.n, chunk_rows)]
        cnt = torch.tensor([len(lst)], dtype=torch.int64, device=dev)
        shuffle.all_reduce_(cnt, "max", w)
        lst += [(srcs[side][0], 0, 0)] * (int(cnt.item()) - len(lst))
        sched.append(lst)
    budget = runner.ctx._props.get("HbmBudgetBytes")
    grace = GR.GraceHashJoin(w, L["stride_in"], L["key_off"], 8,
                             {"O": -(-n_tot[0] // W), "I": -(-n_tot[1] // W)}, chunk_rows,
                             hbm_budget=budget, build=names[build], proj=L["proj"])
    import time
    t0 = time.perf_counter()
    try:
        for side in (0, 1):
            keep = (lay["ko"] if side == 0 else lay["ki"], lay["vo"] if side == 0 else lay["vi"])
            for s, a, b in sched[side]:
                rows = s.chunk(a, b, dev)
                if not L["direct"]:
                    kf, vf = keep
                    rows = torch.stack([rows[:, kf], rows[:, vf if vf is not None else kf]], 1).contiguous()
                grace.add_chunk(names[side], rows.view(torch.uint8).reshape(b - a, -1))
        grace.finish_partitioning()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        acc = torch.zeros(3, dtype=torch.int64, device=dev)          # matches, probe sum, build sum
        bname, pname = names[build], names[1 - build]
        col_b = L["col_o"] if build == 0 else L["col_i"]
        col_p = L["col_i"] if build == 0 else L["col_o"]
        if not (grace.join_sum_all(bname, pname, col_b, col_p, acc)
                or grace.join_sum_hybrid(bname, pname, col_b, col_p, acc)):
            for _, lr, rr in grace.buckets(bname, pname):
                GR.join_sum(lr, rr, grace.key_off, 8, col_b, col_p, acc, grace.table, grace.log_cap)
        cnt, s_probe, s_build = acc.tolist()
        t2 = time.perf_counter()
        stats = grace.stats
    finally:
        grace.release()
    # the device sums are int64: exact only while matches x max |value| < 2^63 per side (the
    # reference's checked Sum throws on overflow).  Decided collectively, so every rank declines
    # together and the compiled stages (whose Sum detects overflow) take over.
    big = torch.tensor([0], dtype=torch.int64, device=dev)
    for side, f in ((0, lay["vo"]), (1, lay["vi"])):
        if f is not None and cnt * max((_max_abs(x, f, dev) for x in srcs[side]), default=0) >= (1 << 63):
            big.fill_(1)
    shuffle.all_reduce_(big, "max", w)
    if int(big.item()):
        raise OverflowError("fused join: int64 sums could overflow for these values")
    s_o, s_i = (s_build, s_probe) if build == 0 else (s_probe, s_build)
    total = lay["co"] * s_o + lay["ci"] * s_i + lay["const"] * cnt
    runner.join_stats = dict(spilled_bytes=stats.spilled_bytes, buckets=stats.buckets, resident=stats.resident,
                             in_hbm=stats.in_hbm, radix_overflow=stats.radix_overflow, build=names[build],
                             layout="projection" if L["direct"] else "key+value rows", matches=cnt,
                             partition_s=round(t1 - t0, 4), join_s=round(t2 - t1, 4))
    kind = desc["agg"]["kind"]
    # the rank's whole result goes to its first Join partition, the others hold empty partials
    if kind in ("Count", "LongCount"):
        res = [[cnt]] + [[0]] * (len(parts) - 1)
    elif kind == "Average":
        res = [[(total, cnt)]] + [[(0, 0)]] * (len(parts) - 1)
    else:
        res = [[total]] + [[0]] * (len(parts) - 1)
    return dict(zip(parts, res))


def _max_abs(src, f, dev) -> int:
    """Bound on |value| of field f of a row source: the generator's value contract (keys below
    ``keys``, payloads 31-bit), or a device min/max pass over a resident column."""
    if isinstance(src, _GenRows):
        return max(src.nk, 1 << 31)
    from ..gpu import stats
    lo, hi = stats.bounds([src.t.cols[src.fields[f]]])[0]
    return max(abs(lo), abs(hi))


def vote(desc, runner):
    """Collective: every rank's layout; fused iff all ranks can and agree."""
    lay = plan_local(desc, runner)
    # one tensor all-gather of (ok, digest of the layout): every rank fused alike, no pickles
    agree, _ = shuffle.vote(lay is not None, sorted(lay.items()) if lay is not None else None, runner.world)
    return lay if agree else None
