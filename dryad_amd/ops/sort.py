"""Sort / partition / gather operators over HBM-resident tensors (HIP kernels in csrc/kernels/sort.hip).

Data model: a *sort entry* array is an ``int64`` tensor of shape ``[n, 2]`` whose rows are the
16-byte ``E128`` structs of the kernels: column 0 = ``lo``, column 1 = ``hi``.  The composite key
is ``(hi << 64) | lo`` compared unsigned; the row index of the record lives in the low 32 bits
of ``lo`` (key-pointer sort).  Fixed-width record tables are ``uint8`` tensors ``[n, stride]``.
"""
from __future__ import annotations

import ctypes
import threading

import torch

from . import _lib
from ._lib import c_u32, c_u64, ptr, stream_of  # noqa: F401

_WS_CACHE: dict = {}


def _workspace(n: int, device) -> torch.Tensor:
    nbytes = int(_lib.lib().dr_sort_u128_workspace(c_u64(max(n, 1))))
    key = (device, nbytes)
    ws = _WS_CACHE.get(key)
    if ws is None:
        # keep one workspace per (device, size); small (<= 1 MiB)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _WS_CACHE.clear()
        _WS_CACHE[key] = ws
    return ws


def empty_entries(n: int, device) -> torch.Tensor:
    return torch.empty((n, 2), dtype=torch.int64, device=device)


def sort_entries(entries: torch.Tensor, begin_bit: int, end_bit: int,
                 tmp: torch.Tensor | None = None) -> torch.Tensor:
    """Stable LSD radix sort of E128 entries on composite bits [begin_bit, end_bit).

    Returns the tensor holding the sorted entries (``entries`` or ``tmp``)."""
    _lib.require_gpu_tensor(entries, "sort_entries")
    n = entries.shape[0]
    if n == 0 or begin_bit >= end_bit:
        return entries
    if tmp is None:
        tmp = torch.empty_like(entries)
    assert tmp.shape[0] >= n
    ws = _workspace(n, entries.device)
    flag = ctypes.c_int(0)
    _lib.call("dr_sort_u128", ptr(entries), ptr(tmp), c_u64(n), begin_bit, end_bit, ptr(ws),
              stream_of(entries), ctypes.byref(flag))
    return tmp[:n] if flag.value else entries


def tie_fixup(entries: torch.Tensor, max_run: int = 4096) -> bool:
    """Re-order runs of equal ``hi`` by ``lo`` (see dr_tie_fixup).  Returns False on overflow."""
    flag = torch.zeros(1, dtype=torch.int32, device=entries.device)
    _lib.call("dr_tie_fixup", ptr(entries), c_u64(entries.shape[0]), c_u32(max_run), ptr(flag), stream_of(entries))
    return int(flag.item()) == 0


def sort_entries_prefix(entries: torch.Tensor, begin_bit: int, tmp: torch.Tensor | None = None) -> torch.Tensor:
    """Sort on composite bits [begin_bit, 128) by sorting hi (bits 64..127) and fixing ties on lo.

    Equivalent to ``sort_entries(entries, begin_bit, 128)`` (stable), two passes cheaper for
    keys with 9-12 bytes when the first 8 key bytes are mostly distinct; falls back to the full
    sort when long runs of equal prefixes exist."""
    if begin_bit >= 64:
        return sort_entries(entries, begin_bit, 128, tmp)
    if tmp is None:
        tmp = torch.empty_like(entries)
    backup = None
    srt = sort_entries(entries, 64, 128, tmp)
    if tie_fixup(srt):
        return srt
    # long equal-prefix runs: redo with the full key width from the (now prefix-sorted) entries;
    # a stable LSD sort over [begin_bit, 64) then [64, 128) restores the exact order
    other = tmp if srt is entries else entries
    out = sort_entries(srt, begin_bit, 64, other[: srt.shape[0]])
    return sort_entries(out, 64, 128, (srt if out is not srt else other)[: srt.shape[0]])


def hi_range(entries: torch.Tensor) -> tuple[int, int]:
    """(min, max) of the unsigned ``hi`` words (one streaming pass)."""
    r = torch.tensor([-1, 0], dtype=torch.int64, device=entries.device)
    _lib.call("dr_hi_range", ptr(entries), c_u64(entries.shape[0]), ptr(r), stream_of(entries))
    mn, mx = r.cpu().tolist()
    return mn & _M64, mx & _M64


_M64 = (1 << 64) - 1
# expected run length the segmented phase is sized for (window = smallest multiple of 8 bits with
# n / 2^window <= RUN_TARGET); overridable for tuning
RUN_TARGET = 16


def _mask_words(begin_bit: int, end_bit: int) -> tuple[int, int]:
    m = ((1 << end_bit) - 1) ^ ((1 << begin_bit) - 1)
    return (m >> 64) & _M64, m & _M64


def _i64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def sort_entries_hybrid(entries: torch.Tensor, begin_bit: int, end_bit: int = 128,
                        tmp: torch.Tensor | None = None, hi_bounds: tuple[int, int] | None = None,
                        stats: dict | None = None) -> torch.Tensor:
    """Stable sort on composite bits [begin_bit, end_bit) = LSD radix on only the top window of
    *varying* key bits + an in-LDS segmented sort of the resulting short runs.

    Bits of ``hi`` above the common prefix of all keys (from ``hi_bounds`` = a known (min, max)
    of hi, e.g. the range-partition separators, or one dr_hi_range pass) are skipped; the window
    is the smallest multiple of 8 bits making the expected run <= RUN_TARGET for uniform keys
    (3 passes for 1e9 keys vs 10 for a full 80-bit TeraSort key).  Skewed keys (a run longer than
    the LDS window) fall back to the full LSD sort of the remaining bits — same result."""
    n = entries.shape[0]
    if n < 2 or begin_bit >= end_bit:
        return entries
    if tmp is None:
        tmp = torch.empty_like(entries)
    if end_bit < 128:   # bits above end_bit are not key bits: no prefix information
        return sort_entries(entries, begin_bit, end_bit, tmp)
    mn, mx = hi_bounds if hi_bounds is not None else hi_range(entries)
    P = 64 - (mn ^ mx).bit_length()            # common prefix of every hi word
    top = 128 - P                              # composite bits >= top are constant
    if top <= begin_bit:
        return entries                         # all keys equal: stable order = input order
    win = 8
    while win < 64 and n > RUN_TARGET << win:
        win += 8
    span = top - begin_bit
    if span <= win + 8 or top - win < 64:
        # few varying bits (or the window would leave hi): plain LSD over the varying bits
        e_ = min(128, begin_bit + ((span + 7) // 8) * 8)
        b = e_ - ((span + 7) // 8) * 8
        if stats is not None:
            stats["path"] = "lsd"
        return sort_entries(entries, b, e_, tmp)
    srt = sort_entries(entries, top - win, top, tmp)
    mh, ml = _mask_words(begin_bit, end_bit)
    flag = torch.zeros(1, dtype=torch.int32, device=entries.device)
    _lib.call("dr_seg_sort_runs", ptr(srt), c_u64(n), top - win - 64, c_u64(mh), c_u64(ml), ptr(flag),
              stream_of(srt))
    if int(flag.item()) == 0:
        if stats is not None:
            stats["path"] = f"hybrid win={win} top={top}"
        return srt
    if stats is not None:
        stats["path"] = "fallback"
    other = tmp if srt is entries else entries
    return sort_entries(srt, begin_bit, 128, other[:n])


def partition_pass(entries: torch.Tensor, shift: int, out: torch.Tensor | None = None):
    """One stable counting-sort pass on the byte digit at ``shift``.

    Returns ``(out, starts)`` where ``starts`` is a device int64 tensor of 257 digit offsets."""
    _lib.require_gpu_tensor(entries, "partition_pass")
    n = entries.shape[0]
    if out is None:
        out = torch.empty_like(entries)
    starts = torch.empty(257, dtype=torch.int64, device=entries.device)
    ws = _workspace(n, entries.device)
    _lib.call("dr_partition_pass_u128", ptr(entries), ptr(out), c_u64(n), shift, ptr(ws), ptr(starts),
              stream_of(entries))
    return out, starts


def extract_keys(rows: torch.Tensor, key_off: int, key_len: int, idx_base: int = 0,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Build E128 sort entries from the byte-string key of fixed-width rows (memcmp order)."""
    _lib.require_gpu_tensor(rows, "extract_keys")
    assert rows.dtype == torch.uint8 and rows.dim() == 2
    n, stride = rows.shape
    if out is None:
        out = empty_entries(n, rows.device)
    _lib.call("dr_extract_keys", ptr(rows), c_u64(n), c_u32(stride), c_u32(key_off), c_u32(key_len),
              c_u32(idx_base), ptr(out), stream_of(rows))
    return out[:n]


def gather_rows(rows: torch.Tensor, entries: torch.Tensor | None = None, index: torch.Tensor | None = None,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = rows[idx(i)] with idx from the low 32 bits of ``entries[i].lo`` or from ``index``."""
    _lib.require_gpu_tensor(rows, "gather_rows")
    assert rows.dtype == torch.uint8 and rows.dim() == 2 and rows.shape[1] % 4 == 0
    src = entries if entries is not None else index
    n = src.shape[0]
    if index is not None:
        assert index.dtype == torch.int64 and index.is_contiguous()
    if out is None:
        out = torch.empty((n, rows.shape[1]), dtype=torch.uint8, device=rows.device)
    _lib.call("dr_gather_rows", ptr(rows), ptr(out), ptr(entries), ptr(index), c_u64(n), c_u32(rows.shape[1]),
              stream_of(rows))
    return out[:n]


def range_dest(entries: torch.Tensor, separators: torch.Tensor, lo_mask: int, descending: bool = False,
               out: torch.Tensor | None = None, subs: int = 1, ranks: int = 1) -> torch.Tensor:
    """Replace entries[i].hi by its destination partition (count of separators before the key).

    With ``subs`` > 1 the ``ranks * subs`` key ranges are renumbered sub-range-major
    (range ``r * subs + b`` -> ``b * ranks + r``): one partition pass then lays out round ``b`` of a
    pipelined exchange as a contiguous, destination-ordered block."""
    _lib.require_gpu_tensor(entries, "range_dest")
    n = entries.shape[0]
    if out is None:
        out = entries
    nsep = separators.shape[0]
    _lib.call("dr_range_dest_u128", ptr(entries), ptr(out), c_u64(n), ptr(separators), c_u32(nsep),
              c_u64(lo_mask & 0xFFFFFFFFFFFFFFFF), int(descending), c_u32(subs), c_u32(ranks), stream_of(entries))
    return out


def bucket_scatter_rows(entries: torch.Tensor, rows: torch.Tensor, out: torch.Tensor, sync: bool = True):
    """Stable scatter of fixed-width ``rows`` into bucket order, bucket = low byte of
    ``entries[i].hi`` (row i <-> entry i), into ``out``.  Returns the 257 bucket start offsets
    (host list; ``sync=False``: the device int64 tensor, no host synchronisation).  One coalesced
    LDS-staged pass over the rows (dr_bucket_scatter_rows) instead of a partition pass of the
    entries plus a row gather through them."""
    _lib.require_gpu_tensor(rows, "bucket_scatter_rows")
    assert rows.dtype == torch.uint8 and rows.dim() == 2 and out.shape[0] >= rows.shape[0]
    n, stride = rows.shape
    if stride % 4 or stride > 128:
        part, starts = partition_pass(entries[:n], 64)
        gather_rows(rows, entries=part, out=out[:n])
        return starts.tolist() if sync else starts
    starts = torch.empty(257, dtype=torch.int64, device=rows.device)
    ws = _workspace(n, rows.device)
    _lib.call("dr_bucket_scatter_rows", ptr(entries), ptr(rows), ptr(out), c_u64(n), c_u32(stride), ptr(ws),
              ptr(starts), stream_of(rows))
    return starts.tolist() if sync else starts


def entries_to_key_int(entries: torch.Tensor, lo_keep_bits: int = 64):
    """Host helper for tests: composite keys as Python ints (hi<<64 | lo masked)."""
    e = entries.cpu().numpy()
    mask = ((1 << lo_keep_bits) - 1) << (64 - lo_keep_bits) if lo_keep_bits < 64 else (1 << 64) - 1
    out = []
    for lo, hi in e.tolist():
        out.append(((hi & (2**64 - 1)) << 64) | ((lo & (2**64 - 1)) & mask))
    return out


# ---------------------------------------------------------------------------------------------
# Compact row sort: 8-byte (32-bit key window, 32-bit row) entries + run fix-up in the row gather
# (csrc/kernels/sort.hip dr_extract_keys64 / dr_sort_u64 / dr_gather_fixup).
_lib.register_signatures({
    "dr_extract_keys64": (ctypes.c_int, [ctypes.c_void_p, c_u64, c_u32, c_u32, c_u32, c_u32, c_u32, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "dr_sort_u64": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_u64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "dr_gather_fixup": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_u64, c_u32, c_u32, c_u32,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dr_gather_fixup_pitch128": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_u64, c_u32, c_u32,
                                                c_u32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dr_rekey64": (ctypes.c_int, [ctypes.c_void_p, c_u32, c_u32, c_u32, c_u32, ctypes.c_void_p, c_u64, ctypes.c_void_p]),
    "dr_e64_position_window": (ctypes.c_int, [ctypes.c_void_p, c_u64, ctypes.c_void_p]),
    "dr_sort_u64_onesweep_workspace": (c_u64, [c_u64]),
    "dr_sort_u64_onesweep": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_u64, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p, c_u64, ctypes.c_void_p, c_u32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
})
# expected entries per run the compact sort sizes its window for (window = smallest multiple of 8
# bits, at most 32, with n <= RUN_TARGET64 * 2^window)
RUN_TARGET64 = 1.0
COMPACT_SORT = True


def common_prefix_bits(mn: int, mx: int) -> int:
    """Leading bits shared by every 64-bit value in [mn, mx]."""
    return 64 - ((mn ^ mx) & _M64).bit_length()


def extract_keys64(rows: torch.Tensor, key_off: int, key_len: int, prefix_bits: int,
                   out: torch.Tensor) -> torch.Tensor:
    """E64 entries (int64 [n]): key bits [prefix_bits, prefix_bits + 32) << 32 | row index."""
    _lib.require_gpu_tensor(rows, "extract_keys64")
    n, stride = rows.shape
    _lib.call("dr_extract_keys64", ptr(rows), c_u64(n), c_u32(stride), c_u32(key_off), c_u32(key_len),
              c_u32(prefix_bits), c_u32(0), ptr(out), stream_of(rows))
    return out[:n]


def window_bits64(n: int) -> int:
    win = 8
    while win < 32 and n > RUN_TARGET64 * (1 << win):
        win += 8
    return win


# E64 sorts of at least this many entries take the single-histogram look-back sort
# (dr_sort_u64_onesweep: one histogram read for all passes instead of a count read per pass)
ONESWEEP_MIN = 1 << 20
_OS_CACHE: dict = {}


def _onesweep_workspace(n: int, device) -> torch.Tensor:
    """Workspace of the look-back sort (granules: 2 KB per 4096-entry tile, ~625 MB at 1.25e9),
    kept per device and grown on demand."""
    nbytes = int(_lib.lib().dr_sort_u64_onesweep_workspace(c_u64(max(n, 1))))
    ws = _OS_CACHE.get(device)
    if ws is None or ws.numel() < nbytes:
        _OS_CACHE.pop(device, None)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _OS_CACHE[device] = ws
    return ws


def lookback_error() -> torch.Tensor:
    """A fresh device flag for ``sort_entries64(err=...)`` (int32 [1], zero)."""
    return torch.zeros(1, dtype=torch.int32, device=torch.cuda.current_device())


_GEN_HIST: dict = {}
_GEN_HIST_LOCK = threading.Lock()


def gen_hist_buffer(parts: int, device) -> torch.Tensor:
    """Per-workgroup [4][256] window-digit histograms a producer of E64 entries writes (int32).
    A buffer of its own per producer call: two jobs on one device never share one."""
    return torch.empty(parts * 1024, dtype=torch.int32, device=device)


def note_gen_hist(keys: torch.Tensor, n: int, part: torch.Tensor | None) -> None:
    """Record that ``part`` holds the window histograms of ``keys[:n]`` (None: forget them).  The
    record keeps ``keys`` alive, so its address cannot be reused by other entries meanwhile."""
    k = (keys.device, keys.data_ptr())
    with _GEN_HIST_LOCK:
        if part is None:
            _GEN_HIST.pop(k, None)
            return
        _GEN_HIST[k] = (keys, n, part)
        while len(_GEN_HIST) > 8:                 # producers whose sort never came: drop the oldest
            _GEN_HIST.pop(next(iter(_GEN_HIST)))


def take_gen_hist(e: torch.Tensor):
    """The producer histograms of the entries ``e`` if they are still the generated ones (one use)."""
    with _GEN_HIST_LOCK:
        h = _GEN_HIST.pop((e.device, e.data_ptr()), None)
    if h is not None and h[1] == e.shape[0]:
        return h[2]
    return None


def sort_entries64(e: torch.Tensor, tmp: torch.Tensor, win: int, gen_hist: torch.Tensor | None = None,
                   err: torch.Tensor | None = None, lookback: bool = True) -> torch.Tensor:
    """Stable LSD sort of E64 entries on their top ``win`` window bits.  ``gen_hist``: the window
    digit histograms of ``e``'s 32-bit key window written by its producer (take_gen_hist).

    At least ONESWEEP_MIN entries take the look-back sort unless ``lookback`` is False (then, like
    smaller sorts, the count + scatter passes).  A look-back sort can fail (a spin gave up, or the
    histograms do not count the entries): it then ORs a non-zero code into ``err`` (a device int32
    flag, see lookback_error; required for look-back sorts) and leaves the entries unsorted and
    reordered, so the caller rebuilds them from the rows and sorts again with ``lookback=False``."""
    n = e.shape[0]
    flag = ctypes.c_int(0)
    if lookback and n >= ONESWEEP_MIN:
        if err is None:
            raise ValueError("sort_entries64: a look-back sort needs an error flag (err=lookback_error())")
        ws = _onesweep_workspace(n, e.device)
        parts = 0 if gen_hist is None else gen_hist.numel() // 1024
        _lib.call("dr_sort_u64_onesweep", ptr(e), ptr(tmp), c_u64(n), 64 - win, 64, ptr(ws), c_u64(ws.numel()),
                  ptr(gen_hist), c_u32(parts), ptr(err), stream_of(e), ctypes.byref(flag))
    else:
        ws = _workspace(n, e.device)
        _lib.call("dr_sort_u64", ptr(e), ptr(tmp), c_u64(n), 64 - win, 64, ptr(ws), stream_of(e), ctypes.byref(flag))
    return tmp[:n] if flag.value else e


def gather_fixup(rows: torch.Tensor, srt: torch.Tensor, out: torch.Tensor, key_off: int, key_len: int,
                 win: int, flag: torch.Tensor, err: torch.Tensor | None = None):
    """Row gather through window-sorted E64 entries with the run fix-up.  ``flag`` (int32) gets
    bit 0 when a run outgrows the window, bit 1 when an entry names a row past ``rows`` (never
    read); ``err``: the look-back sort's error word, when set the kernel reads nothing."""
    n, stride = rows.shape
    _lib.call("dr_gather_fixup", ptr(rows), ptr(out), ptr(srt), c_u64(n), c_u32(stride), c_u32(key_off),
              c_u32(key_len), 64 - win, ptr(flag), ptr(err), stream_of(rows))


def compact_sort_ok(rows: torch.Tensor, key_len: int) -> bool:
    n, stride = rows.shape
    return COMPACT_SORT and 2 <= n < (1 << 32) and stride % 4 == 0 and 1 <= key_len <= 16


def sort_rows_compact(rows: torch.Tensor, out: torch.Tensor, ent: torch.Tensor, tmp: torch.Tensor,
                      key_off: int, key_len: int, hi_bounds: tuple[int, int] | None = None,
                      keys_ready: bool = False, stats: dict | None = None):
    """Stable sort of fixed-width ``rows`` by the byte-string key into ``out[:n]`` through 8-byte
    entries.  ``ent``/``tmp``: int64 scratch of >= n elements each.  ``hi_bounds``: (min, max) of
    the first 8 key bytes (big-endian) of all rows, used to skip their common prefix; with
    ``keys_ready`` ``ent[:n]`` already holds the entries for prefix 0 (fused generator).
    Returns ``out[:n]``, or None when a run of equal windows is too long for the gather's fix-up
    (heavily duplicated keys): the caller then sorts on full keys."""
    n = rows.shape[0]
    if hi_bounds is None:
        e = extract_keys64(rows, key_off, key_len, 0, ent)
        hi_bounds = _hi_range64(e)
        P = common_prefix_bits(hi_bounds[0] & ~0xFFFFFFFF, hi_bounds[1] | 0xFFFFFFFF)
        if P:
            e = extract_keys64(rows, key_off, key_len, P, ent)
    else:
        P = min(common_prefix_bits(*hi_bounds), 8 * key_len)
        if keys_ready and P == 0:
            e = ent[:n]
        else:
            e = extract_keys64(rows, key_off, key_len, P, ent)
    win = min(window_bits64(n), max(8, ((8 * key_len - P + 7) // 8) * 8), 32)
    flags = torch.zeros(2, dtype=torch.int32, device=rows.device)        # [gather overflow, look-back error]
    srt = sort_entries64(e, tmp, win, err=flags[1:])
    gather_fixup(rows, srt, out, key_off, key_len, win, flags[:1], err=flags[1:])
    if stats is not None:
        stats["path"] = f"compact win={win} prefix={P}"
    overflow, failed = (int(x) != 0 for x in flags.tolist())
    if failed:              # the look-back sort failed: the entries again, count + scatter passes
        e = extract_keys64(rows, key_off, key_len, P, ent)
        srt = sort_entries64(e, tmp, win, lookback=False)
        flags.zero_()
        gather_fixup(rows, srt, out, key_off, key_len, win, flags[:1])
        overflow = int(flags[0].item()) != 0
        if stats is not None:
            stats["path"] += " look-back failed: count+scatter"
    if overflow:
        if stats is not None:
            stats["path"] += " overflow"
        return None
    return out[:n]


def _hi_range64(e: torch.Tensor, chunk: int = 1 << 26) -> tuple[int, int]:
    """(min, max) of the E64 window words, as hi-word bounds (window bits in the top 32).  Chunked,
    so the temporaries stay at 2 x 512 MB however large ``e`` is (a 1.25e9-entry table next to a
    290 GB sort working set has no room for a full-size copy)."""
    mins, maxs = [], []
    for a in range(0, e.shape[0], chunk):
        w = (e[a:a + chunk] >> 32) & 0xFFFFFFFF          # unsigned window (>> is arithmetic on int64)
        mins.append(w.min())
        maxs.append(w.max())
    mn, mx = int(torch.stack(mins).min().item()), int(torch.stack(maxs).max().item())
    return mn << 32, mx << 32


_lib.register_signatures({
    "dr_extract_keys64_tile_parts": (c_u32, [c_u64]),
    "dr_extract_keys64_tile": (ctypes.c_int, [ctypes.c_void_p, c_u64, c_u32, c_u32, c_u32, c_u32, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]),
})


def extract_keys64_tile(rows: torch.Tensor, key_off: int, key_len: int, prefix_bits: int, out: torch.Tensor,
                        hist: bool = False):
    """``extract_keys64`` reading whole rows through LDS (dr_extract_keys64_tile); ``hist``: also
    the window-digit histograms a following look-back sort takes instead of its histogram read.
    Returns (entries, histograms or None)."""
    _lib.require_gpu_tensor(rows, "extract_keys64_tile")
    n = rows.shape[0]
    stride = rows.stride(0) if n > 1 else rows.shape[1]     # (a [n, rec] view of 128-byte-pitch rows)
    assert rows.stride(1) == 1 and key_off + key_len <= rows.shape[1]
    part = None
    if hist and n >= ONESWEEP_MIN:
        part = gen_hist_buffer(int(_lib.lib().dr_extract_keys64_tile_parts(c_u64(n))), rows.device)
    _lib.call("dr_extract_keys64_tile", ptr(rows), c_u64(n), c_u32(stride), c_u32(key_off), c_u32(key_len),
              c_u32(prefix_bits), ptr(out), ptr(part), stream_of(rows))
    return out[:n], part


# ------------------------------------------------------------------------------------------------
# Rows at a 128-byte pitch.  A table whose 100-byte records each start an aligned 128-byte line
# (bytes 100..127 padding) costs 28% more bytes to write, but every random row read of the sort's
# gather is then ONE HBM line instead of ~1.78 (the fetch unit is the whole 128-byte line): at
# 1e9 rows the gather drops from 57.9 to 43.6 ms and the generator grows from 15.4 to 19.1 ms
# (profiles/r3/pitch128_ab.log).  Used for gen://terasort tables that only a one-rank OrderBy reads.
PITCH = 128


def gather_fixup_pitch128(rows_p: torch.Tensor, srt: torch.Tensor, out: torch.Tensor, key_off: int, key_len: int,
                          win: int, flag: torch.Tensor, err: torch.Tensor | None = None):
    """gather_fixup from ``rows_p`` ([n, 128] uint8: the first 100 bytes of each row are the record)
    into ``out`` ([n, 100], back to back)."""
    n = rows_p.shape[0]
    if rows_p.shape[1] != PITCH or out.shape[1] != 100 or not rows_p.is_contiguous():
        raise ValueError("gather_fixup_pitch128: [n, 128] input rows and [n, 100] output rows")
    _lib.call("dr_gather_fixup_pitch128", ptr(rows_p), ptr(out), ptr(srt), c_u64(n), c_u32(100), c_u32(key_off),
              c_u32(key_len), 64 - win, ptr(flag), ptr(err), stream_of(rows_p))


def rekey64(rows: torch.Tensor, ent: torch.Tensor, key_off: int, key_len: int, P: int) -> torch.Tensor:
    """ent[i] := key bits [P, P + 32) of row (ent[i] & 0xFFFFFFFF) << 32 | row (rows [m, pitch])."""
    _lib.require_gpu_tensor(rows, "rekey64")
    _lib.call("dr_rekey64", ptr(rows), c_u32(rows.shape[1]), c_u32(key_off), c_u32(key_len), c_u32(P), ptr(ent),
              c_u64(ent.shape[0]), stream_of(rows))
    return ent


def _sort64_into(e: torch.Tensor, tmp: torch.Tensor, win: int, gen_hist=None, err=None,
                 lookback: bool = True) -> torch.Tensor:
    """sort_entries64 whose result always ends in ``e`` (``tmp`` may alias the gather's output)."""
    srt = sort_entries64(e, tmp, win, gen_hist, err=err, lookback=lookback)
    if srt.data_ptr() != e.data_ptr():
        e.copy_(srt)
    return e


# One-rank sorts of pitch-128 tables: the entries sorted on their top BUCKET_BITS window bits only
# (three look-back passes instead of four) and every run of equal 24-bit prefixes -- a key bucket
# of ~n / 2^24 rows -- ordered by the row gather itself (dr_gather_bucket_pitch128), when the
# buckets average BUCKET_MIN_ROWS .. BUCKET_MAX_ROWS rows (the gather's window holds runs of up
# to 192 rows; a longer one is flagged and the full-key chain below takes over)
BUCKET_BITS = 24
BUCKET_MIN_ROWS, BUCKET_MAX_ROWS = 16, 96


def bucket_sort_ok(n: int, key_len: int) -> bool:
    return 8 * key_len > BUCKET_BITS and key_len <= 16 and \
        (BUCKET_MIN_ROWS << BUCKET_BITS) <= n <= min(BUCKET_MAX_ROWS << BUCKET_BITS, (1 << 32) - 1)


def sort_rows_pitch128(rows_p: torch.Tensor, out: torch.Tensor, keys: torch.Tensor, key_off: int, key_len: int,
                       keys_ready: bool = True, stats: dict | None = None, keys_fmt: str = "e64") -> torch.Tensor:
    """Stable sort of the records in ``rows_p`` ([n, 128], 100-byte records) by their byte-string
    key into ``out[:n]`` ([>= n, 100]).  ``keys[:n]``: the rows' compact entries for prefix 0
    (written by the generator) when ``keys_ready``, else the key is read from the rows.  The radix
    sort's ping-pong buffer is ``out`` itself (free until the gather), so the working set is rows
    + output + 8 bytes per row.

    A run of equal 32-bit windows too long for the gather's fix-up (heavily duplicated keys) is
    resolved exactly without more memory: an LSD chain of compact sorts over every 32-bit window
    of the key, from the least significant, each window re-read from the rows (``rekey64``),
    then a gather without fix-up.

    ``keys_fmt`` "e64@out": the producer wrote the entries into ``out``'s first n * 8 bytes (the
    bucket sort's home for them: its odd pass count then ends in ``keys``, see bucket_sort_ok)."""
    n = rows_p.shape[0]
    if n == 0:
        return out[:0]
    if n >= (1 << 32) or key_len > 16 or key_off + key_len > 100:
        raise ValueError("sort_rows_pitch128: < 2^32 rows, key inside the 100-byte record, <= 16 bytes")
    tmp = out.view(-1)[: n * 8].view(torch.int64)
    e = keys[:n]
    in_out = keys_ready and keys_fmt == "e64@out"
    gen_hist = take_gen_hist(tmp if in_out else e) if keys_ready else None
    flags = torch.zeros(2, dtype=torch.int32, device=rows_p.device)      # [gather overflow, look-back error]
    flag = flags[:1]
    path = "compact pitch128"
    lookback = True
    bucket = keys_ready and key_off == 0 and bucket_sort_ok(n, key_len)
    if in_out and not bucket:
        e.copy_(tmp)                            # the entries where the four-pass path wants them
    if bucket:
        src, dst = (tmp, e) if in_out else (e, tmp)
        srt = sort_entries64(src, dst, BUCKET_BITS, gen_hist, err=flags[1:])
        if srt.data_ptr() != e.data_ptr():
            e.copy_(srt)                        # the entries must not lie under the output
        _lib.call("dr_gather_bucket_pitch128", ptr(rows_p), ptr(out), ptr(e), c_u64(n), c_u32(key_off),
                  c_u32(key_len), 64 - BUCKET_BITS, ptr(flag), ptr(flags[1:]), stream_of(rows_p))
        path += (" gen-hist" if gen_hist is not None and n >= ONESWEEP_MIN else "") + \
            f" bucket sort: win={BUCKET_BITS} + in-LDS bucket order"
        overflow, failed = (int(x) != 0 for x in flags.tolist())
        chain = overflow or failed
        if failed:
            lookback = False
            path += " look-back failed"
    elif keys_ready and key_off == 0:
        win = min(window_bits64(n), max(8, ((8 * key_len + 7) // 8) * 8), 32)
        _sort64_into(e, tmp, win, gen_hist, err=flags[1:])
        if gen_hist is not None and n >= ONESWEEP_MIN:
            path += " gen-hist"
        gather_fixup_pitch128(rows_p, e, out[:n], key_off, key_len, win, flag, err=flags[1:])
        path += f" win={win}"
        overflow, failed = (int(x) != 0 for x in flags.tolist())
        chain = overflow or failed
        if failed:          # the entries are lost: rebuilt from the rows by the chain below
            lookback = False
            path += " look-back failed"
    else:
        torch.arange(n, out=e)                  # entries = row index; windows come from the rows
        chain = True
    if chain:
        bits = 8 * key_len
        windows = list(range(max(0, bits - 32), -1, -32))
        if windows[-1] != 0:
            windows.append(0)
        if not lookback:
            torch.arange(n, out=e)
        flags.zero_()
        for P in windows:                       # least significant window first
            rekey64(rows_p, e, key_off, key_len, P)
            _sort64_into(e, tmp, 32, err=flags[1:], lookback=lookback)
        _lib.call("dr_e64_position_window", ptr(e), c_u64(n), stream_of(e))
        gather_fixup_pitch128(rows_p, e, out[:n], key_off, key_len, 32, flag, err=flags[1:])
        if int(flags[1].item()) != 0:           # a look-back pass of the chain failed: once more without
            torch.arange(n, out=e)
            for P in windows:
                rekey64(rows_p, e, key_off, key_len, P)
                _sort64_into(e, tmp, 32, lookback=False)
            _lib.call("dr_e64_position_window", ptr(e), c_u64(n), stream_of(e))
            gather_fixup_pitch128(rows_p, e, out[:n], key_off, key_len, 32, flag)
            path += " (look-back failed: count+scatter)"
        path += f" + full-key LSD chain over windows {windows}"
    if stats is not None:
        stats["path"] = path
    return out[:n]
