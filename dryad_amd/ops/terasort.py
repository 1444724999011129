"""TeraSort record store kernels: synthetic generator + valsort-style checker (csrc/kernels/terasort.hip)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import c_u32, c_u64, ptr, stream_of

_lib.register_signatures({
    "dr_ts_sample_keys": (ctypes.c_int, [c_u64, c_u64, c_u64, c_u64, c_u64, c_u64, ctypes.c_void_p, ctypes.c_void_p]),
    "dr_terasort_gen_gather": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_u64, c_u64, c_u64, ctypes.c_void_p]),
})

RECORD_BYTES = 100
KEY_BYTES = 10
# lo-word mask that keeps the two key bytes stored in lo (bits 63..48) and drops the row index.
LO_KEY_MASK_10 = 0xFFFF000000000000


def generate(out: torch.Tensor, first_index: int, seed: int) -> torch.Tensor:
    """Fill ``out`` ([n, 100] uint8, HBM) with records first_index .. first_index+n-1."""
    _lib.require_gpu_tensor(out, "terasort.generate")
    assert out.dtype == torch.uint8 and out.dim() == 2 and out.shape[1] == RECORD_BYTES
    _lib.call("dr_terasort_gen", ptr(out), c_u64(out.shape[0]), c_u64(first_index), c_u64(seed & (2**64 - 1)),
              stream_of(out))
    _lib.written(out)
    return out


def generate_with_keys(out: torch.Tensor, first_index: int, seed: int, keys: torch.Tensor,
                       hi_range: torch.Tensor | None = None) -> torch.Tensor:
    """``generate`` fused with key extraction: ``keys`` ([n, 2] int64) receives the sort entries
    ``extract_keys(out, 0, 10)`` would build, ``hi_range`` ([2] int64, initialised to [-1, 0])
    the unsigned min/max of their hi words.  Saves the extraction pass of a following sort."""
    _lib.require_gpu_tensor(out, "terasort.generate_with_keys")
    n = out.shape[0]
    assert keys.shape[0] >= n and keys.dtype == torch.int64 and keys.is_contiguous()
    _lib.call("dr_terasort_gen_keys", ptr(out), c_u64(n), c_u64(first_index), c_u64(seed & (2**64 - 1)),
              ptr(keys), c_u32(0), ptr(hi_range), stream_of(out))
    return out


def generate_with_keys64(out: torch.Tensor, first_index: int, seed: int, keys: torch.Tensor,
                         hi_range: torch.Tensor | None = None) -> torch.Tensor:
    """``generate`` fused with the 8-byte entries of the compact row sort (key bytes 0..3 << 32 |
    row index, ``keys`` int64 [>= n]) and the min/max of the key's first 8 bytes."""
    _lib.require_gpu_tensor(out, "terasort.generate_with_keys64")
    n = out.shape[0]
    assert keys.numel() >= n and keys.dtype == torch.int64 and keys.is_contiguous()
    _lib.call("dr_terasort_gen_keys64", ptr(out), c_u64(n), c_u64(first_index), c_u64(seed & (2**64 - 1)),
              ptr(keys), c_u32(0), ptr(hi_range), stream_of(out))
    return out


def generate_with_keys64_pitch128(out: torch.Tensor, first_index: int, seed: int, keys: torch.Tensor,
                                  hi_range: torch.Tensor | None = None, hist: bool = False) -> torch.Tensor:
    """``generate_with_keys64`` with the records at a 128-byte pitch (``out`` [n, 128] uint8, bytes
    100..127 of each row zero): one aligned HBM line per record (ops/sort.sort_rows_pitch128).
    ``hist``: the generator also writes the digit histograms of the entries' key window, handed to
    the sort of ``keys[:n]`` (ops/sort.take_gen_hist) so that it skips its histogram read."""
    from . import sort as S
    _lib.require_gpu_tensor(out, "terasort.generate_with_keys64_pitch128")
    n = out.shape[0]
    assert out.shape[1] == 128 and keys.numel() >= n and keys.dtype == torch.int64 and keys.is_contiguous()
    part = None
    if hist and n >= S.ONESWEEP_MIN:
        parts = int(_lib.lib().dr_terasort_gen_hist_parts(c_u64(n)))
        part = S.gen_hist_buffer(parts, out.device)
    _lib.call("dr_terasort_gen_keys64_pitch128", ptr(out), c_u64(n), c_u64(first_index), c_u64(seed & (2**64 - 1)),
              ptr(keys), c_u32(0), ptr(hi_range), ptr(part), stream_of(out))
    S.note_gen_hist(keys, n, part)
    return out


def check(rows: torch.Tensor, acc: torch.Tensor | None = None, descending: bool = False) -> torch.Tensor:
    """Accumulate [sum of record hashes mod 2^64, #adjacent order violations] into ``acc``
    (``descending``: violations of the descending order)."""
    _lib.require_gpu_tensor(rows, "terasort.check")
    if acc is None:
        acc = torch.zeros(2, dtype=torch.int64, device=rows.device)
    _lib.call("dr_terasort_check_desc" if descending else "dr_terasort_check", ptr(rows), c_u64(rows.shape[0]),
              ptr(acc), stream_of(rows))
    return acc


def sample_keys(first: int, seed: int, off: int, stride: int, m: int, lo_or: int, device) -> torch.Tensor:
    """Sort entries ([m, 2] int64, the ``generate_keys_only`` layout with ``lo_or`` OR-ed into lo)
    of records ``first + off + k * stride`` (k < m), generated at those positions only: the
    sampler of a distributed sort over gen://terasort draws them without a full entry table."""
    out = torch.empty((max(m, 0), 2), dtype=torch.int64, device=device)
    if m > 0:
        _lib.call("dr_ts_sample_keys", c_u64(first), c_u64(seed & (2**64 - 1)), c_u64(off), c_u64(stride), c_u64(m),
                  c_u64(lo_or & (2**64 - 1)), ptr(out), stream_of(out))
    return out


def gen_gather(out: torch.Tensor, idx: torch.Tensor, first: int, seed: int) -> torch.Tensor:
    """``out[p]`` := record ``first + idx[p]`` (``out`` [m, 100] uint8 rows back to back, ``idx``
    int32 [m] slice offsets): the send-buffer pack of a distributed sort over gen://terasort."""
    _lib.require_gpu_tensor(out, "terasort.gen_gather")
    m = idx.shape[0]
    assert out.dtype == torch.uint8 and out.shape[0] >= m and out.shape[1] == RECORD_BYTES and out.is_contiguous()
    assert idx.dtype == torch.int32 and idx.is_contiguous()
    _lib.call("dr_terasort_gen_gather", ptr(out), ptr(idx), c_u64(m), c_u64(first), c_u64(seed & (2**64 - 1)),
              stream_of(out))
    return out[:m]


_lib.register_signatures({
    "dr_terasort_gen_gather64": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_u64, c_u64, c_u64, ctypes.c_void_p,
                                                c_u32, ctypes.c_void_p]),
    "dr_terasort_gen_entries64": (ctypes.c_int, [ctypes.c_void_p, c_u64, c_u64, c_u64, c_u32, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
    "dr_ts_fine_starts": (ctypes.c_int, [ctypes.c_void_p, c_u64, c_u32, ctypes.c_void_p, ctypes.c_void_p]),
    "dr_ts_tile_merge": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, c_u32, c_u32, c_u32, ctypes.c_void_p, ctypes.c_void_p]),
    "dr_ts_tile_cap": (ctypes.c_uint32, []),
})


def gen_entries64(keys: torch.Tensor, first: int, seed: int, hist: bool = True):
    """E64 sort entries of records ``first .. first + n - 1`` (``keys`` int64 [n]: key bytes 0..3
    << 32 | i), no records; with ``hist`` also the window-digit histograms a following look-back
    sort of ``keys`` takes (ops/sort.sort_entries64 gen_hist).  Returns the histograms or None."""
    from . import sort as S
    _lib.require_gpu_tensor(keys, "terasort.gen_entries64")
    n = keys.shape[0]
    assert keys.dtype == torch.int64 and keys.dim() == 1 and n < (1 << 32)
    part = None
    if hist and n >= S.ONESWEEP_MIN:
        part = S.gen_hist_buffer(int(_lib.lib().dr_terasort_gen_hist_parts(c_u64(n))), keys.device)
    _lib.call("dr_terasort_gen_entries64", ptr(keys), c_u64(n), c_u64(first), c_u64(seed & (2**64 - 1)), c_u32(0),
              ptr(part), stream_of(keys))
    return part


def gen_gather64(out: torch.Tensor, ent: torch.Tensor, first: int, seed: int, seg: torch.Tensor | None = None,
                 n: int | None = None) -> torch.Tensor:
    """``out[p]`` := record ``first + (ent[q] & 0xFFFFFFFF)`` (``ent`` int64 sorted E64 entries),
    q = p, or with ``seg`` (device int64 [nseg, 2] of {out row, entry}, ascending, seg[0, 0] = 0,
    nseg <= 64) q = seg[s, 1] + p - seg[s, 0] for the last segment starting at or before p; ``n``
    rows (default ``ent``'s length)."""
    _lib.require_gpu_tensor(out, "terasort.gen_gather64")
    m = ent.shape[0] if n is None else n
    assert out.dtype == torch.uint8 and out.shape[0] >= m and out.shape[1] == RECORD_BYTES and out.is_contiguous()
    assert ent.dtype == torch.int64 and ent.is_contiguous()
    nseg = 0
    if seg is not None:
        assert seg.dtype == torch.int64 and seg.is_contiguous() and seg.dim() == 2 and seg.shape[1] == 2
        nseg = seg.shape[0]
    _lib.call("dr_terasort_gen_gather64", ptr(out), ptr(ent), c_u64(m), c_u64(first), c_u64(seed & (2**64 - 1)),
              ptr(seg), c_u32(nseg), stream_of(out))
    return out[:m]


def fine_starts(ent: torch.Tensor, fb: int) -> torch.Tensor:
    """int32 [2^fb + 1]: for each fine bucket k (the top ``fb`` key bits) the first position of the
    window-sorted entries ``ent`` in bucket >= k."""
    _lib.require_gpu_tensor(ent, "terasort.fine_starts")
    starts = torch.empty((1 << fb) + 1, dtype=torch.int32, device=ent.device)
    _lib.call("dr_ts_fine_starts", ptr(ent), c_u64(ent.shape[0]), c_u32(fb), ptr(starts), stream_of(ent))
    return starts


def tile_cap() -> int:
    """Rows of one fine bucket the receive side orders in LDS (ts_tile_merge)."""
    return int(_lib.lib().dr_ts_tile_cap())


def tile_merge(rows: torch.Tensor, out: torch.Tensor, pre: torch.Tensor, cnt: torch.Tensor, outoff: torch.Tensor,
               fb: int, overflow: torch.Tensor, key_off: int = 0, key_len: int = 10, descending: bool = False) -> None:
    """Order the received fine buckets: bucket k's rows are the W slices ``rows[pre[s, k] :
    pre[s, k] + cnt[s, k]]`` (all sharing their top ``fb`` key bits), written in key order (ties by
    source, then slice position) to ``out[outoff[k]:]``.  The key is the ``key_len`` <= 10 bytes at
    byte ``key_off`` (memcmp order; its bits inverted with ``descending``, matching entries whose
    window was inverted).  A bucket past tile_cap() rows is left out and flags ``overflow``."""
    W, K = cnt.shape
    assert pre.shape == (W, K) and pre.dtype == torch.int64 and cnt.dtype == torch.int32 and outoff.shape == (K,)
    rec = rows.shape[1]
    # rows of any width (a multiple of 4 bytes, 12..128)
    assert out.shape[1] == rec and rec % 4 == 0 and 12 <= rec <= 128 and rows.stride(0) == rec
    assert 1 <= key_len <= 10 and 0 <= key_off and key_off + key_len <= rec
    _lib.call("dr_ts_tile_merge_w", ptr(rows), ptr(out), ptr(pre.contiguous()), ptr(cnt.contiguous()),
              ptr(outoff.contiguous()), c_u32(W), c_u32(K), c_u32(fb), ptr(overflow), c_u32(rec),
              c_u32(key_off), c_u32(key_len), c_u32(int(bool(descending))), stream_of(rows))
    _lib.written(out)


def bucket_copy(rows: torch.Tensor, out: torch.Tensor, pre: torch.Tensor, cnt: torch.Tensor,
                outoff: torch.Tensor) -> None:
    """tile_merge for fine buckets that each hold ONE key (no key bit below the bucket bits):
    bucket k's W slices ``rows[pre[s, k] : pre[s, k] + cnt[s, k]]`` copied in source order to
    ``out[outoff[k]:]``, whatever the bucket's size (runs of equal keys past tile_cap())."""
    W, K = cnt.shape
    rec = rows.shape[1]
    assert pre.shape == (W, K) and pre.dtype == torch.int64 and cnt.dtype == torch.int32 and outoff.shape == (K,)
    assert out.shape[1] == rec and rec % 4 == 0 and rows.stride(0) == rec and out.stride(0) == rec
    _lib.call("dr_ts_bucket_copy", ptr(rows), ptr(out), ptr(pre.contiguous()), ptr(cnt.contiguous()),
              ptr(outoff.contiguous()), c_u32(W), c_u32(K), c_u32(rec), stream_of(rows))
    _lib.written(out)


_lib.register_signatures({
    "dr_ts_bucket_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, c_u32, c_u32, c_u32, ctypes.c_void_p]),
    "dr_ts_pack_rows_w": (ctypes.c_int, [ctypes.c_void_p, c_u64, c_u32, ctypes.c_void_p, c_u64, ctypes.c_void_p,
                                         c_u32, ctypes.c_void_p, c_u32, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "dr_ts_tile_merge_w": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, c_u32, c_u32, c_u32, ctypes.c_void_p, c_u32,
                                          c_u32, c_u32, c_u32, ctypes.c_void_p]),
})


def pack_rows(out: torch.Tensor, rows: torch.Tensor, ent: torch.Tensor, n: int, seg: torch.Tensor | None = None,
              err: torch.Tensor | None = None, bad: torch.Tensor | None = None) -> torch.Tensor:
    """Send rows of a materialised table: ``out[p]`` := ``rows[ent[q(p)] & 0xFFFFFFFF]`` for p < n
    (``rows`` [n_in, rec] or [n_in, 128] uint8 holding rec-byte records, rec a multiple of 4 in
    8..128, ``out`` [>= n, rec]);
    q(p) = p, or through ``seg`` (device int64 [nseg <= 256, 2] of {out row, entry}, ascending,
    seg[0, 0] = 0).  ``err``: the look-back sort's error word (nothing is read when it is set);
    ``bad`` (int32 [1]) is set when an entry names a row past n_in.  Returns ``bad``."""
    _lib.require_gpu_tensor(out, "terasort.pack_rows")
    pitch = rows.stride(0)
    rec = out.shape[1]
    assert rows.dtype == torch.uint8 and pitch in (rec, 128) and rows.stride(1) == 1
    assert rec % 4 == 0 and 8 <= rec <= 128 and rows.shape[1] >= rec
    assert out.dtype == torch.uint8 and out.is_contiguous() and out.shape[0] >= n
    assert ent.dtype == torch.int64 and ent.is_contiguous()
    nseg = 0
    if seg is not None:
        assert seg.dtype == torch.int64 and seg.is_contiguous() and seg.dim() == 2 and seg.shape[1] == 2
        nseg = seg.shape[0]
        assert nseg <= 256
    else:
        assert ent.shape[0] >= n
    if bad is None:
        bad = torch.zeros(1, dtype=torch.int32, device=out.device)
    _lib.call("dr_ts_pack_rows_w", ptr(rows), c_u64(rows.shape[0]), c_u32(pitch), ptr(ent), c_u64(n), ptr(seg),
              c_u32(nseg), ptr(out), c_u32(rec), ptr(err), ptr(bad), stream_of(out))
    _lib.written(out)
    return bad
