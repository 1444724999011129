"""Device text operators (csrc/kernels/text.hip): line splitting and WordCount tokenisation.

A partition's text lives in HBM as one byte heap; lines and tokens are (offset, length) int64
pairs.  Whitespace = ' ', '\\t', '\\r', '\\n' (String.Split() with no arguments, which is what the
reference's WordCount sample uses)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import relational as R
from . import sort as S
from ._lib import c_u64, ptr, stream_of, vp, c_i32

_lib.register_signatures({
    "dr_text_marks": (c_i32, [vp, c_u64, vp, vp]),
    "dr_token_hash": (c_i32, [vp, vp, vp, c_u64, vp, vp]),
    "dr_token_verify": (c_i32, [vp, vp, vp, vp, c_u64, vp, vp]),
    "dr_str_match": (c_i32, [vp, vp, vp, c_u64, vp, ctypes.c_int64, c_i32, vp, vp]),
})

MATCH_EQ, MATCH_PREFIX, MATCH_SUFFIX, MATCH_CONTAINS = 0, 1, 2, 3


def str_match(heap, off, ln, pattern: str, mode: int) -> torch.Tensor:
    """Boolean mask of strings (heap, off, len) that equal / start with / end with / contain
    ``pattern`` (UTF-8 byte comparison, i.e. ordinal string semantics)."""
    n = off.shape[0]
    out = torch.empty(n, dtype=torch.bool, device=off.device)
    pat = pattern.encode("utf-8")
    pt = torch.frombuffer(bytearray(pat), dtype=torch.uint8).to(off.device) if pat else \
        torch.zeros(1, dtype=torch.uint8, device=off.device)
    if heap.numel() == 0:
        heap = torch.zeros(1, dtype=torch.uint8, device=off.device)
    _lib.call("dr_str_match", ptr(heap), ptr(off.contiguous()), ptr(ln.contiguous()), c_u64(n), ptr(pt),
              ctypes.c_int64(len(pat)), mode, ptr(out), stream_of(off))
    return out

SPACE = b" \t\r\n"


def marks(buf: torch.Tensor) -> torch.Tensor:
    _lib.require_gpu_tensor(buf, "text.marks")
    m = torch.empty(buf.shape[0], dtype=torch.uint8, device=buf.device)
    _lib.call("dr_text_marks", ptr(buf), c_u64(buf.shape[0]), ptr(m), stream_of(buf))
    return m


def lines(buf: torch.Tensor, m: torch.Tensor | None = None):
    """(offset, length) of every line ('\\n', '\\r\\n' or '\\r' separated, Appendix C)."""
    n = buf.shape[0]
    if n == 0:
        z = torch.empty(0, dtype=torch.int64, device=buf.device)
        return z, z
    m = marks(buf) if m is None else m
    st = torch.nonzero(m & 1, as_tuple=False).flatten()
    nxt = torch.cat([st[1:], torch.tensor([n], dtype=torch.int64, device=buf.device)])
    ln = nxt - st
    # strip the terminator: "\n", "\r\n" or a lone "\r" (the last line may have none)
    last = buf[(nxt - 1).clamp_min(0)]
    term = ((last == 10) | (last == 13)).to(torch.int64)
    prev = buf[(nxt - 2).clamp_min(0)]
    term = term + ((last == 10) & (prev == 13) & (ln >= 2)).to(torch.int64)
    ln = ln - term
    return st, ln


def tokens(buf: torch.Tensor, m: torch.Tensor | None = None):
    """(offset, length) of every whitespace-separated token, in text order."""
    if buf.shape[0] == 0:
        z = torch.empty(0, dtype=torch.int64, device=buf.device)
        return z, z
    m = marks(buf) if m is None else m
    st = torch.nonzero(m & 2, as_tuple=False).flatten()
    en = torch.nonzero(m & 4, as_tuple=False).flatten()
    return st, en - st + 1


def token_hash(buf, off, ln) -> torch.Tensor:
    out = torch.empty(off.shape[0], dtype=torch.int64, device=buf.device)
    _lib.call("dr_token_hash", ptr(buf), ptr(off.contiguous()), ptr(ln.contiguous()), c_u64(off.shape[0]), ptr(out),
              stream_of(buf))
    return out


def gather_strings(buf: torch.Tensor, off: torch.Tensor, ln: torch.Tensor) -> list:
    """Host strings for (offset, length) pairs (one ragged device gather + one copy)."""
    if off.numel() == 0:
        return []
    tot = int(ln.sum().item())
    base = torch.repeat_interleave(off, ln)
    starts = torch.cumsum(ln, 0) - ln
    pos = base + (torch.arange(tot, device=buf.device) - torch.repeat_interleave(starts, ln))
    data = buf.index_select(0, pos).cpu().numpy().tobytes()
    lens = ln.cpu().tolist()
    out, p = [], 0
    for L in lens:
        out.append(data[p:p + L].decode("utf-8", errors="replace"))
        p += L
    return out


def _word_groups(buf: torch.Tensor):
    """Token groups of ``buf``: (token offsets, lengths, sorted representative token per group,
    group start positions in the sorted order, token count), or None on a 64-bit hash collision
    between different words."""
    off, ln = tokens(buf)
    nt = off.shape[0]
    if nt == 0:
        return off, ln, None, None, 0
    h = token_hash(buf, off, ln)
    e = torch.empty((nt, 2), dtype=torch.int64, device=buf.device)
    e[:, 1] = h
    e[:, 0] = torch.arange(nt, dtype=torch.int64, device=buf.device)
    srt = S.sort_entries_hybrid(e, 64)
    seg, nseg, starts = R.segment_ids(srt, 0)
    order = srt[:, 0] & 0xFFFFFFFF
    rep_sorted = order.index_select(0, starts).index_select(0, seg)      # representative per sorted token
    rep = torch.empty_like(rep_sorted)
    rep[order] = rep_sorted
    bad = torch.zeros(1, dtype=torch.int32, device=buf.device)
    _lib.call("dr_token_verify", ptr(buf), ptr(off), ptr(ln), ptr(rep), c_u64(nt), ptr(bad), stream_of(buf))
    if int(bad.item()):
        return None
    return off, ln, order.index_select(0, starts), starts, nt


def word_count(buf: torch.Tensor) -> list:
    """[(word, count)] of the whitespace tokens in ``buf`` (device hash-group + exact check)."""
    g = _word_groups(buf)
    if g is None:
        # 64-bit hash collision between different words: exact host path (never seen in practice)
        from collections import Counter
        off, ln = tokens(buf)
        return list(Counter(gather_strings(buf, off, ln)).items())
    off, ln, reps, starts, nt = g
    if nt == 0:
        return []
    ends = torch.cat([starts[1:], torch.tensor([nt], dtype=torch.int64, device=buf.device)])
    counts = (ends - starts).cpu().tolist()
    words = gather_strings(buf, off.index_select(0, reps), ln.index_select(0, reps))
    return list(zip(words, counts))


def word_count_table(buf: torch.Tensor):
    """The (word, count) groups of ``buf`` as an HBM table of (String, Int32) tuples -- the words
    compacted into a string heap on the device, no host round trip -- or None when the exact
    check found a hash collision (the caller then takes the host path)."""
    from ..gpu.table import DeviceTable, Shape
    from . import channel as CH
    g = _word_groups(buf)
    if g is None:
        return None
    off, ln, reps, starts, nt = g
    if nt == 0:
        return None
    ends = torch.cat([starts[1:], torch.tensor([nt], dtype=torch.int64, device=buf.device)])
    counts = ends - starts
    wl = ln.index_select(0, reps)
    heap, woff = CH.compact_heap(buf, off.index_select(0, reps), wl)
    cnt = counts.to(torch.int32) if nt < (1 << 31) else counts
    t = DeviceTable.from_columns({"Item1": woff, "Item1#len": wl, "Item2": cnt}, Shape("tuple", ["Item1", "Item2"]))
    t.strs = {"Item1": heap}
    return t


_lib.register_signatures({
    "dr_scatter_strings": (c_i32, [vp, vp, vp, c_u64, vp, c_u64, ctypes.c_uint32, ctypes.c_uint32, vp, vp]),
})


def scatter_strings(heap: torch.Tensor, off: torch.Tensor, ln: torch.Tensor, dst: torch.Tensor, dst_off: int,
                    max_len: int | None = None) -> bool:
    """Copy string i (``heap[off[i]: off[i] + ln[i]]``) into row i of ``dst`` ([n, stride] uint8)
    at byte ``dst_off``.  Returns False when a string is longer than ``max_len`` (default: the
    room up to the row's end), which is then cut."""
    n, stride = dst.shape
    ml = stride - dst_off if max_len is None else max_len
    flag = torch.zeros(1, dtype=torch.int32, device=dst.device)
    if heap.numel() == 0:
        heap = torch.zeros(8, dtype=torch.uint8, device=dst.device)
    _lib.call("dr_scatter_strings", ptr(heap), ptr(off.to(torch.int64).contiguous()), ptr(ln.to(torch.int64).contiguous()),
              c_u64(n), ptr(dst), c_u64(stride), ctypes.c_uint32(dst_off), ctypes.c_uint32(ml), ptr(flag),
              stream_of(dst))
    return int(flag.item()) == 0
